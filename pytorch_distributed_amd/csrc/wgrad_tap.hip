// Tap-reuse weight gradient of 3x3 stride-1 pad-1 convolutions for gfx950 (MI355X).
//
//   dW[co][r][s][ci] = sum over output pixels p of dY[p][co] * X[p + (r-1, s-1)][ci]
//
// The generic implicit-GEMM weight gradient (csrc/conv_gemm.hip WGRAD) gathers its B operand per
// (tap, channel) column tile, so every N-tile re-reads X for its taps and dY for its rows: at the
// layer1 3x3 (64 -> 64, 56x56, batch 400) a launch reads 1.6 GB for 0.32 GB of operands
// (profiles/pmc_r5_step.md). Here a block owns a range of pixels and ALL nine taps of a 64 x 64
// (co, ci) tile: every dY and X byte of the range is loaded once, and the nine taps read the same
// LDS image of X at nine row offsets.
//
// Padded pixel space: pixel rows are indexed as q = (n, y + 1, x + 1) in an image padded by one
// pixel on every side (Hp = H + 2, Wp = W + 2), with dY and X zero at the padding positions. Tap
// (r, s) is then a constant row shift d = (r - 1) Wp + (s - 1) of the X image for EVERY q -- no
// per-element boundary masks -- at (Hp Wp) / (H W) extra MFMA work (1.07x at 56, 1.15x at 28).
//
// Block = 512 threads (8 waves, one block per CU), its padded-row range [q0, q0 + KB) in steps of
// 64 rows. LDS: X in a 512-row ring (64 channels = 128-B rows, chunks XOR-swizzled by row as the
// COL images of conv_gemm.hip), dY in NS + 1 tile slots [64 rows][64 co]. Operands arrive by
// LDS-DMA (buffer_load ... lds; padding and out-of-range rows as out-of-bounds offsets, which
// write zeros), NS = 4 steps ahead, one counted vmcnt + one barrier per step. The BN+ReLU operand
// prologue of a PRE-BatchNorm X is applied in LDS to the rows the NEXT step adds, between the
// barrier and this step's MFMAs (no wave of this step reads those rows; the next barrier publishes
// them), with the 64 channels' coefficients staged in LDS once. MFMA 16x16x32
// with swapped operands (D = X_frag x dY_frag^T): each lane ends with 4 consecutive (ci) columns of
// one co row, stored as f32x4 into the split-K slab [split][Cout][9 Cin] that pda_wgrad_reduce sums.
// Wave (wr, wc): co rows 32 wr .. +32, columns 144 wc .. +144 of the 576 = 9 taps x 64 ci.
#include "common.h"

namespace {

constexpr int WT_NT = 512;
constexpr int WT_NS = 4;            // steps in flight
constexpr int WT_RING = 512;        // X ring rows (power of two)
constexpr int WT_SLAB = WT_RING * 128;
constexpr int WT_ATILE = 64 * 128;  // dY tile [64 rows][64 co]
constexpr int WT_COEF = 64 * 2 * 4;  // BN scale / shift of the block's 64 input channels (f32)
constexpr int WT_LDS = WT_SLAB + (WT_NS + 1) * WT_ATILE + WT_COEF;

struct WtParams {
  const void* dy;      // [Nb, H, W, Cout] 16-bit
  const void* x;       // [Nb, H, W, Cin] 16-bit (PRE-BatchNorm when pro_sc is set)
  float* slab;         // [splits][Cout][9 Cin]
  const float* pro_sc; const float* pro_sh;   // optional BN+ReLU applied to X (channel Cin)
  int Nb, H, W, Cin, Cout;
  int Hp, Wp, Kp;      // padded geometry, Kp = Nb Hp Wp
  int kb;              // padded rows per block (multiple of 64)
  int nsteps;          // kb / 64
  int halo;            // Wp + 1
  int co_tiles, ci_tiles;
  FastDiv dHpWp, dWp;
};

typedef dma_rsrc_t wt_rsrc_t;
__device__ __forceinline__ wt_rsrc_t wt_rsrc(const void* base, uint32_t bytes) { return dma_rsrc(base, bytes); }
__device__ __forceinline__ void wt_dma16(wt_rsrc_t r, char* lds, uint32_t voff) { dma16_asm(r, lds, voff); }
template <int N> __device__ __forceinline__ void wt_vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// chunk swizzle of a 64-column (128-B) k-major row, conv_gemm.hip col_swz<64>: conflict-free
// transposed fragment reads for ANY row offset (rows r .. r+3, r+8 .. r+11 of a read fall on 8
// distinct (row parity, swizzle) classes for every r)
__device__ __forceinline__ int wt_swz(int row) { return (((row >> 1) & 1) << 1) | (((row >> 3) & 1) << 2); }

constexpr uint32_t WT_OOB = 0x80000000u;

template <int DT, bool PRO>
__global__ __launch_bounds__(WT_NT, 1) void wgrad_tap_kernel(WtParams p_arg) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) WtParams KP;
  KP& p = *(KP*)__builtin_amdgcn_kernarg_segment_ptr();
#else
  const WtParams& p = p_arg;
#endif
  __shared__ __attribute__((aligned(16))) char smem[WT_LDS];
  char* slab = smem;
  char* atl = smem + WT_SLAB;
  float* coef = reinterpret_cast<float*>(smem + WT_SLAB + (WT_NS + 1) * WT_ATILE);   // [2][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid & 1, wc = wid >> 1;
  const int ntile = p.co_tiles * p.ci_tiles;
  const int lt = (int)xcd_remap(blockIdx.x, gridDim.x);   // the tiles of one split share an XCD
  const int split = lt / ntile, tile = lt - split * ntile;
  const int cot = tile / p.ci_tiles, cit = tile - cot * p.ci_tiles;
  // padded row q -> byte offset of element c_elems of its pixel in an NHWC tensor of C channels, or
  // OOB for padding / out-of-range rows
  const FastDiv dHpWp = p.dHpWp, dWp = p.dWp;
  const int Kp = p.Kp, H = p.H, W = p.W;
  auto wt_pix = [&](int q, int C, int c_elems) __attribute__((always_inline)) -> uint32_t {
    if (q < 0 || q >= Kp) return WT_OOB;
    const uint32_t n = fdiv((uint32_t)q, dHpWp), rem = (uint32_t)q - n * dHpWp.d;
    const uint32_t yp = fdiv(rem, dWp), xp = rem - yp * dWp.d;
    if (yp < 1 || yp > (uint32_t)H || xp < 1 || xp > (uint32_t)W) return WT_OOB;
    return ((((n * H + yp - 1) * W + xp - 1) * (uint32_t)C) + (uint32_t)c_elems) * 2u;
  };
  const int q0 = split * p.kb;
  const int q_end = min(q0 + p.kb, p.Kp);
  const int ns = p.nsteps;
  const wt_rsrc_t rdy = wt_rsrc(p.dy, (int)((uint32_t)p.Nb * p.H * p.W * p.Cout * 2u));
  const wt_rsrc_t rx = wt_rsrc(p.x, (int)((uint32_t)p.Nb * p.H * p.W * p.Cin * 2u));

  // X rows: step s reads [q0 + 64 s - halo, q0 + 64 s + 64 + halo); rows are issued in 8-row
  // pieces from the 8-aligned base b0; fr(s) = first row not needed by steps <= s (8-aligned)
  const int b0 = (q0 - p.halo) & ~7;
  auto fr = [&](int s) { return (q0 + 64 * (s + 1) + p.halo + 7) & ~7; };
  const int lrow = lane >> 3, lch = lane & 7;
  // one 8-row X piece starting at row r (8-aligned): lane -> row r + lrow, physical chunk lch
  auto x_piece = [&](int r, bool live) __attribute__((always_inline)) {
    const int row = r + lrow;
    const int lc = lch ^ wt_swz(row);
    wt_dma16(rx, slab + (r & (WT_RING - 1)) * 128, live ? wt_pix(row, p.Cin, cit * 64 + lc * 8) : WT_OOB);
  };
  // the dY tile of step s, piece w: rows q0 + 64 s + 8 w + lrow (rows past the range: zero)
  auto a_piece = [&](int s, int w) __attribute__((always_inline)) {
    const int rl = 8 * w + lrow;
    const int q = q0 + 64 * s + rl;
    const int lc = lch ^ wt_swz(rl);
    const uint32_t off = q < q_end ? wt_pix(q, p.Cout, cot * 64 + lc * 8) : WT_OOB;
    wt_dma16(rdy, atl + (s % (WT_NS + 1)) * WT_ATILE + 8 * w * 128, off);
  };
  // prologue: issue the operands of steps 0 .. NS-1, in step order (step 0 carries the X rows
  // [b0, fr(0)), every later step the 64 rows [fr(s-1), fr(s)) and its dY tile). The counted
  // waits below only ever leave YOUNGER groups in flight, so the size of the step-0 group (which
  // differs between waves) never enters a count.
  for (int r = b0 + 8 * wid; r < fr(0); r += 64) x_piece(r, true);
  a_piece(0, wid);
#pragma unroll
  for (int s = 1; s < WT_NS; ++s) {
    x_piece(fr(s - 1) + 8 * wid, s < ns);
    a_piece(s, wid);
  }
  // BN+ReLU in LDS of the X rows [r_lo, r_hi) (padding rows stay 0): one 16-B chunk per thread
  // per 64 rows; the coefficients of the block's 64 channels come from LDS
  auto pro_rows = [&](int r_lo, int r_hi) __attribute__((always_inline)) {
    if constexpr (PRO) {
      for (int rr = r_lo + (tid >> 3); rr < r_hi; rr += WT_NT / 8) {
        if (wt_pix(rr, p.Cin, 0) == WT_OOB) continue;
        const int lc = lch ^ wt_swz(rr);
        i32x4* cp = reinterpret_cast<i32x4*>(slab + (rr & (WT_RING - 1)) * 128 + lch * 16);
        i32x4 v = *cp;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const f32x2 sc = *reinterpret_cast<const f32x2*>(coef + lc * 8 + 2 * k);
          const f32x2 sh = *reinterpret_cast<const f32x2*>(coef + 64 + lc * 8 + 2 * k);
          const f32x2 u = unpack2<DT>((uint32_t)v[k]);
          const f32x2 f = f32x2{fmaxf(__builtin_fmaf(u.x, sc.x, sh.x), 0.f),
                                fmaxf(__builtin_fmaf(u.y, sc.y, sh.y), 0.f)};
          v[k] = (int)pack2<DT>(f);
        }
        *cp = v;
      }
    }
  };
  if constexpr (PRO) {
    if (tid < 64) {
      coef[tid] = p.pro_sc[cit * 64 + tid];
      coef[64 + tid] = p.pro_sh[cit * 64 + tid];
    }
    // step 0's rows: landed (every wave's step-0 group), then transformed before the loop's first
    // barrier publishes them
    wt_vm_wait<2 * (WT_NS - 1)>();
    __syncthreads();
    pro_rows(b0, fr(0));
  }

  f32x4 acc[2][9];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // per column tile j of the wave: tap row shift and channel base (wave-uniform)
  int dsh[9], cb[9];
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int col = wc * 144 + 16 * j;
    const int t = col >> 6;
    dsh[j] = (t / 3 - 1) * p.Wp + (t % 3 - 1);
    cb[j] = col & 63;
  }
  const int g = lane >> 4, fi = lane & 15, fq = fi >> 2, fp = fi & 3;
  // Fragment addresses, precomputed per lane (the transposed reads of frag_col, conv_gemm.hip):
  // lane reads rows L, L + 4 (L = 8g + fq) of a 32-row substep, 8 bytes at column chunk
  // cbase/8 + fp/2 (+ 8 B for odd fp). X rows of tap shift d at step s, substep s2 are
  // q0 + 64 s + 32 s2 + d + L: the ring row advances by 32 per substep, and as 32 = 0 mod 16 the
  // row swizzle (bits 1 and 3) is the same at every step -- so each address is its step-0 value
  // plus (64 s + 32 s2) * 128 B, wrapped at the 64 KiB ring: one add and one and per address.
  const int L0 = 8 * g + fq;
  const int half = (fp & 1) << 3;
  int xa[9][2];    // X: ring byte offset at s = s2 = 0, rows L0 / L0 + 4
#pragma unroll
  for (int j = 0; j < 9; ++j)
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int r = q0 + dsh[j] + L0 + 4 * h;
      const int chunk = cb[j] / 8 + (fp >> 1);
      xa[j][h] = (r & (WT_RING - 1)) * 128 + ((chunk ^ wt_swz(r)) << 4) + half;
    }
  int aa[2][2][2];   // dY tile: byte offset of substep s2, co tile i, row L0 / L0 + 4
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = s2 * 32 + L0 + 4 * h;
        const int chunk = (wr * 32 + 16 * i) / 8 + (fp >> 1);
        aa[s2][i][h] = k * 128 + ((chunk ^ wt_swz(k)) << 4) + half;
      }

  for (int s = 0; s < ns; ++s) {
    // step s's operands have landed -- with the prologue, step s+1's too (it transforms them now)
    if constexpr (PRO) wt_vm_wait<2 * (WT_NS - 2)>();
    else wt_vm_wait<2 * (WT_NS - 1)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the operands of step s + NS (past the range: out-of-bounds no-ops, so the count per step
    // stays 2 per wave); their slots were last read in step s - 1
    x_piece(fr(s + WT_NS - 1) + 8 * wid, s + WT_NS < ns);
    a_piece(s + WT_NS, wid);
    // BN+ReLU of the rows step s+1 adds: nothing in step s reads them (rows >= fr(s))
    if (s + 1 < ns) pro_rows(fr(s), fr(s + 1));
    const char* sa = atl + (s % (WT_NS + 1)) * WT_ATILE;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 fa[2], fb[9];
#pragma unroll
      for (int i = 0; i < 2; ++i) {   // dY: rows s2*32 + L0 (+4) of the tile, co column
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, sa + aa[s2][i][0]));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, sa + aa[s2][i][1]));
        fa[i] = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
      const int roff = (64 * s + 32 * s2) * 128;
#pragma unroll
      for (int j = 0; j < 9; ++j) {   // X: ring rows of the tap shift, this step and substep
        const int a0 = (xa[j][0] + roff) & (WT_SLAB - 1);
        const int a1 = (xa[j][1] + roff) & (WT_SLAB - 1);
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, slab + a0));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, slab + a1));
        fb[j] = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
      __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 9; ++j) acc[i][j] = mfma16<DT>(fb[j], fa[i], acc[i][j]);
      __builtin_amdgcn_s_setprio(0);
    }
  }
  wt_vm_wait<0>();   // the trailing no-op DMAs, before the block can exit

  // slab[split][co][t * Cin + ci]: lane = co row (lane & 15) of tile i, 4 consecutive columns
  const size_t N = 9 * (size_t)p.Cin;
  float* out = p.slab + (size_t)split * p.Cout * N;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int co = cot * 64 + wr * 32 + 16 * i + fi;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int col = wc * 144 + 16 * j;
      const int t = col >> 6;
      const int ci = cit * 64 + (col & 63) + 4 * g;
      *reinterpret_cast<f32x4*>(out + (size_t)co * N + (size_t)t * p.Cin + ci) = acc[i][j];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// The stem's weight gradient in the tap-reuse form (the stem conv = a 4x4 stride-1 conv with pad
// 2 on the 2x2 space-to-depth image: 16 input channels, 64 output channels, 112 x 112), with the
// stem BatchNorm's backward formed in LDS (dY = k1*dz + k2*y + k3, WGRAD_BNA's operand):
//
//   dW[co][r][s][ci] = sum over output pixels p of dY[p][co] * X[p + (r - 2, s - 2)][ci]
//
// Padded index space: output rows q = (n, oy, ox) over an Hp x Wp = (H + 3) x (W + 3) grid (real
// outputs oy, ox < H, W; the rest are padding rows with dY = 0) and X rows q' = (n, yp, xp) with
// X[q'] = x[n][yp - 2][xp - 2] (zero outside). Tap (r, s) is the constant FORWARD row shift
// d = r Wp + s for every q (the forward halo is 3 Wp + 3 rows, none backward).
//
// Block = 512 threads (8 waves: wr = co half, wc = 4 taps = 64 of the 256 columns), one block per
// CU, its padded-row range [q0, q0 + KB) in steps of 64 rows. LDS: X in a 1024-row ring of 32-B
// rows (16 channels), dz and y in NS + 1 tile slots [64 rows][64 co] each; all by LDS-DMA, NS = 4
// steps ahead. X rows sit in 16-row blocks at slot (j & 8) | ((j & 7) ^ 4 (j >> 3)): the transposed
// fragment reads of a wave touch rows L .. L+3 and L+8 .. L+11 (32 B each) in one lane group, and
// the slot map puts them in 8 distinct 32-B bank windows for any row offset L. dY of step s+1 is
// formed in place in its dz slot during step s (its DMA has landed; nothing in step s reads it).
#ifndef PDA_SW_NS
#define PDA_SW_NS 4
#endif
constexpr int SW_NS = PDA_SW_NS;                  // steps in flight
constexpr int SW_RING = 1024;                      // X ring rows (power of two, 16-row blocks)
constexpr int SW_XROW = 32;                        // 16 channels x 2 B
constexpr int SW_XBYTES = SW_RING * SW_XROW;
constexpr int SW_ATILE = 64 * 128;                 // dz / y tile [64 rows][64 co]
constexpr int SW_COEF = 3 * 64 * 4;
constexpr int SW_LDS = SW_XBYTES + 2 * (SW_NS + 1) * SW_ATILE + SW_COEF;

struct SwParams {
  const void* dz;      // [Nb, H, W, 64] 16-bit, the stem BN's masked gradient
  const void* y;       // [Nb, H, W, 64] 16-bit, the BN input
  const float* k;      // [3][64]: dY = k[0] dz + k[1] y + k[2]
  const void* x;       // [Nb, H, W, 16] 16-bit (the space-to-depth image)
  float* slab;         // [splits][64][16 taps x 16]
  int Nb, H, W;
  int Hp, Wp, Kp;
  int kb, nsteps, fhalo;   // fhalo = 3 Wp + 3
  FastDiv dHpWp, dWp;
};

__device__ __forceinline__ int sw_slot(int j) { return (j & 8) | ((j & 7) ^ ((j >> 3) << 2)); }
// ring byte offset of X row r
__device__ __forceinline__ int sw_xaddr(int r) {
  const int rr = r & (SW_RING - 1);
  return ((rr & ~15) + sw_slot(rr & 15)) * SW_XROW;
}

template <int DT>
__global__ __launch_bounds__(WT_NT, 1) void wgrad_stem_tap_kernel(SwParams p_arg) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) SwParams KP;
  KP& p = *(KP*)__builtin_amdgcn_kernarg_segment_ptr();
#else
  const SwParams& p = p_arg;
#endif
  __shared__ __attribute__((aligned(16))) char smem[SW_LDS];
  char* xr = smem;
  char* tz = smem + SW_XBYTES;                               // dz slots (dY after the transform)
  char* ty = tz + (SW_NS + 1) * SW_ATILE;                   // y slots
  float* coef = reinterpret_cast<float*>(ty + (SW_NS + 1) * SW_ATILE);   // [3][64]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid & 1, wc = wid >> 1;
  const int split = (int)xcd_remap(blockIdx.x, gridDim.x);
  const FastDiv dHpWp = p.dHpWp, dWp = p.dWp;
  const int Kp = p.Kp, H = p.H, W = p.W;
  // padded X row q' -> byte offset of its 16-channel pixel (+ c elems), OOB outside the image
  auto x_pix = [&](int q, int c_elems) __attribute__((always_inline)) -> uint32_t {
    if (q < 0 || q >= Kp) return WT_OOB;
    const uint32_t n = fdiv((uint32_t)q, dHpWp), rem = (uint32_t)q - n * dHpWp.d;
    const uint32_t yp = fdiv(rem, dWp), xp = rem - yp * dWp.d;
    if (yp < 2 || yp >= (uint32_t)H + 2 || xp < 2 || xp >= (uint32_t)W + 2) return WT_OOB;
    return ((((n * H + yp - 2) * W + xp - 2) * 16u) + (uint32_t)c_elems) * 2u;
  };
  const int q0 = split * p.kb;
  const int q_end = min(q0 + p.kb, Kp);
  const int ns = p.nsteps;
  const uint32_t npix = (uint32_t)p.Nb * p.H * p.W;
  const wt_rsrc_t rdz = wt_rsrc(p.dz, (int)(npix * 128u));
  const wt_rsrc_t ry = wt_rsrc(p.y, (int)(npix * 128u));
  const wt_rsrc_t rx = wt_rsrc(p.x, (int)(npix * 32u));

  // Every stream of rows below advances by exactly 64 padded rows per call: its (image, y, x)
  // coordinates are tracked incrementally (one fdiv pair at the start, then adds and compares)
  // instead of two fdivs per row per step.
  struct Trk { uint32_t n, y, x; };
  const uint32_t Hp = (uint32_t)p.Hp, Wp = (uint32_t)p.Wp;
  auto trk = [&](int q) __attribute__((always_inline)) -> Trk {
    const uint32_t qq = (uint32_t)max(q, 0);
    const uint32_t n = fdiv(qq, dHpWp), rem = qq - n * dHpWp.d;
    const uint32_t y = fdiv(rem, dWp);
    return Trk{n, y, rem - y * dWp.d};
  };
  const bool wide = Wp > 64;   // (the stem: Wp = 115) at most one wrap per 64 rows: branch-free
  auto adv = [&](Trk& t) __attribute__((always_inline)) {
    t.x += 64;
    if (wide) {
      const bool wx = t.x >= Wp;
      t.x -= wx ? Wp : 0u;
      t.y += wx;
      const bool wy = t.y >= Hp;
      t.y -= wy ? Hp : 0u;
      t.n += wy;
    } else {
      while (t.x >= Wp) { t.x -= Wp; ++t.y; }
      while (t.y >= Hp) { t.y -= Hp; ++t.n; }
    }
  };

  // X rows: step s reads [q0 + 64 s, q0 + 64 s + 64 + fhalo); pieces of 32 rows from the
  // 32-aligned base b0; fr(s) = first row not needed by steps <= s (32-aligned)
  const int b0 = q0 & ~31;
  auto fr = [&](int s) { return (q0 + 64 * (s + 1) + p.fhalo + 31) & ~31; };
  // one 32-row X piece at row r (32-aligned): lane -> slot lane/2 of the piece, channel half lane&1
  const int xb = lane >> 5, xsl = (lane >> 1) & 15;
  auto x_piece = [&](int r, bool live) __attribute__((always_inline)) {
    const int row = r + 16 * xb + sw_slot(xsl);            // (sw_slot is an involution)
    wt_dma16(rx, xr + (r & (SW_RING - 1)) * SW_XROW, live ? x_pix(row, (lane & 1) * 8) : WT_OOB);
  };
  // the pieces after the prologue's bulk: rows fr(0) + 32 wid + ..., 64 further per call
  int xq = fr(0) + 32 * wid + 16 * xb + sw_slot(xsl);
  Trk tx = trk(xq);
  auto x_next = [&](int r, bool live) __attribute__((always_inline)) {
    const bool in = live && xq < Kp && tx.y >= 2 && tx.y < (uint32_t)H + 2 && tx.x >= 2 &&
                    tx.x < (uint32_t)W + 2;
    const uint32_t off = in ? ((((tx.n * H + tx.y - 2) * W + tx.x - 2) * 16u) + (lane & 1) * 8u) * 2u
                            : WT_OOB;
    wt_dma16(rx, xr + (r & (SW_RING - 1)) * SW_XROW, off);
    xq += 64;
    adv(tx);
  };
  // the dz / y tiles of step s, piece w: rows q0 + 64 s + 8 w + lane/8 (rows past the range: zero)
  const int lrow = lane >> 3, lch = lane & 7;
  const int arl = 8 * wid + lrow, alc = lch ^ wt_swz(arl);
  Trk ta = trk(q0 + arl);
  auto a_pieces = [&](int s, int w) __attribute__((always_inline)) {
    const int q = q0 + 64 * s + arl;
    const uint32_t off = q < q_end && ta.y < (uint32_t)H && ta.x < (uint32_t)W
                             ? ((((ta.n * H + ta.y) * W + ta.x) * 64u) + alc * 8u) * 2u : WT_OOB;
    const int slot = (s % (SW_NS + 1)) * SW_ATILE + 8 * w * 128;
    wt_dma16(rdz, tz + slot, off);
    wt_dma16(ry, ty + slot, off);
    adv(ta);
  };
  // per step: waves 0, 1 add the step's two X pieces (3 DMAs), every wave its dz + y pieces (2)
  const bool xw = wid < 2;
  // prologue: steps 0 .. NS-1 in order (step 0 also carries X rows [b0, fr(0)))
  for (int r = b0 + 32 * wid; r < fr(0); r += 256) x_piece(r, true);
  a_pieces(0, wid);
#pragma unroll
  for (int s = 1; s < SW_NS; ++s) {
    if (xw) x_next(fr(s - 1) + 32 * wid, s < ns);
    a_pieces(s, wid);
  }
  if (tid < 192) coef[tid] = p.k[tid];
  // dY = k1 dz + k2 y + k3 in place of step s's dz slot: one 16-B chunk per thread (the same
  // 8 channels at every step: coefficients in registers); padding and out-of-range rows stay 0
  const int frl = tid >> 3, fpc = tid & 7, flc = fpc ^ wt_swz(frl);
  Trk tf = trk(q0 + frl);
  f32x2 K1[4], K2[4], K3[4];
  auto form_dy = [&](int s) __attribute__((always_inline)) {
    const int q = q0 + 64 * s + frl;
    const bool ok = q < q_end && tf.y < (uint32_t)H && tf.x < (uint32_t)W;
    adv(tf);
    const int off = (s % (SW_NS + 1)) * SW_ATILE + frl * 128 + fpc * 16;
    i32x4* zp = reinterpret_cast<i32x4*>(tz + off);
    const i32x4 z = *zp, yv = *reinterpret_cast<const i32x4*>(ty + off);
    i32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const f32x2 d = unpack2<DT>((uint32_t)z[k]), u = unpack2<DT>((uint32_t)yv[k]);
      const f32x2 f = f32x2{__builtin_fmaf(K1[k].x, d.x, __builtin_fmaf(K2[k].x, u.x, K3[k].x)),
                            __builtin_fmaf(K1[k].y, d.y, __builtin_fmaf(K2[k].y, u.y, K3[k].y))};
      o[k] = ok ? (int)pack2<DT>(f) : 0;
    }
    *zp = o;
  };
  // step 0's operands: landed (every wave's step-0 group), formed before the loop's first barrier
  if (xw) wt_vm_wait<3 * (SW_NS - 1)>(); else wt_vm_wait<2 * (SW_NS - 1)>();
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    K1[k] = *reinterpret_cast<const f32x2*>(coef + flc * 8 + 2 * k);
    K2[k] = *reinterpret_cast<const f32x2*>(coef + 64 + flc * 8 + 2 * k);
    K3[k] = *reinterpret_cast<const f32x2*>(coef + 128 + flc * 8 + 2 * k);
  }
  form_dy(0);

  f32x4 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int g = lane >> 4, fi = lane & 15, fq = fi >> 2, fp = fi & 3;
  const int L0 = 8 * g + fq;
  const int half = (fp & 1) << 3;
  // X fragment addresses at s = s2 = 0 for the wave's 4 taps (t = 4 wc + j: shift r Wp + s), rows
  // L0 / L0 + 4; a 32-row substep / 64-row step advances them by 1 / 2 KiB (32 = 0 mod 16 keeps
  // the slot map), wrapped at the ring
  int xa[4][2];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int t = 4 * wc + j;
    const int dsh = (t >> 2) * p.Wp + (t & 3);
#pragma unroll
    for (int h = 0; h < 2; ++h)
      xa[j][h] = sw_xaddr(q0 + dsh + L0 + 4 * h) + ((fp >> 1) << 4) + half;
  }
  int aa[2][2][2];   // dY tile: byte offset of substep s2, co tile i, row L0 / L0 + 4
#pragma unroll
  for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int k = s2 * 32 + L0 + 4 * h;
        const int chunk = (wr * 32 + 16 * i) / 8 + (fp >> 1);
        aa[s2][i][h] = k * 128 + ((chunk ^ wt_swz(k)) << 4) + half;
      }

  for (int s = 0; s < ns; ++s) {
    // steps s and s+1 have landed (s+1 is formed now)
    if (xw) wt_vm_wait<3 * (SW_NS - 2)>(); else wt_vm_wait<2 * (SW_NS - 2)>();
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    // the operands of step s + NS (past the range: out-of-bounds no-ops -- the per-step count
    // stays fixed); their slots were last read in step s - 1
    if (xw) x_next(fr(s + SW_NS - 1) + 32 * wid, s + SW_NS < ns);
    a_pieces(s + SW_NS, wid);
    if (s + 1 < ns) form_dy(s + 1);
    const char* sa = tz + (s % (SW_NS + 1)) * SW_ATILE;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s16x8 fa[2], fb[4];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, sa + aa[s2][i][0]));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, sa + aa[s2][i][1]));
        fa[i] = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
      const int roff = (64 * s + 32 * s2) * SW_XROW;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int a0 = (xa[j][0] + roff) & (SW_XBYTES - 1);
        const int a1 = (xa[j][1] + roff) & (SW_XBYTES - 1);
        const s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, xr + a0));
        const s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, xr + a1));
        fb[j] = s16x8{v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = mfma16<DT>(fb[j], fa[i], acc[i][j]);
    }
  }
  wt_vm_wait<0>();   // the trailing no-op DMAs, before the block can exit

  // slab[split][co][t * 16 + ci]: lane = co row (lane & 15) of tile i, 4 consecutive channels
  float* out = p.slab + (size_t)split * 64 * 256;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int co = wr * 32 + 16 * i + fi;
#pragma unroll
    for (int j = 0; j < 4; ++j)
      *reinterpret_cast<f32x4*>(out + (size_t)co * 256 + (4 * wc + j) * 16 + 4 * g) = acc[i][j];
  }
}

FastDiv wt_div(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

}  // namespace

extern "C" {

// Split-K weight-gradient slabs of a 3x3 / stride-1 / pad-1 convolution, tap-reuse form:
// slab [splits][Cout][9 Cin] (f32) -- pda_wgrad_reduce sums them like the generic kernel's.
// dy [Nb,H,W,Cout], x [Nb,H,W,Cin] 16-bit; pro_sc / pro_sh: BN+ReLU of a PRE-BatchNorm x (or null).
// kb: padded rows per split (multiple of 64); splits = ceil(Nb (H+2)(W+2) / kb). Cin, Cout multiples
// of 64; W <= 59 (the X ring holds 4 steps + the two halos). Returns -2 on a shape it does not take.
int pda_wgrad_tap(const void* dy, const void* x, float* slab, const float* pro_sc,
                  const float* pro_sh, int Nb, int H, int W, int Cin, int Cout, int kb, int splits,
                  int dt, hipStream_t st) {
  if ((Cin % 64) || (Cout % 64) || kb <= 0 || (kb % 64) || W > 59 || H <= 0 || W <= 0)
    return -2;
  if ((pro_sc == nullptr) != (pro_sh == nullptr)) return -2;
  WtParams p{};
  p.dy = dy; p.x = x; p.slab = slab; p.pro_sc = pro_sc; p.pro_sh = pro_sh;
  p.Nb = Nb; p.H = H; p.W = W; p.Cin = Cin; p.Cout = Cout;
  p.Hp = H + 2; p.Wp = W + 2;
  const long long kp = (long long)Nb * p.Hp * p.Wp;
  if (kp >= (1ll << 30) || (long long)Nb * H * W * (Cin > Cout ? Cin : Cout) * 2 >= 0x7fffffffll) return -4;
  p.Kp = (int)kp;
  p.kb = kb; p.nsteps = kb / 64; p.halo = p.Wp + 1;
  if ((long long)splits * kb < kp || (long long)(splits - 1) * kb >= kp) return -3;
  p.co_tiles = Cout / 64; p.ci_tiles = Cin / 64;
  p.dHpWp = wt_div((uint32_t)(p.Hp * p.Wp));
  p.dWp = wt_div((uint32_t)p.Wp);
  const dim3 grid(splits * p.co_tiles * p.ci_tiles);
  const bool pro = pro_sc != nullptr;
  if (dt == DT_BF16) {
    if (pro) TRACKED_LAUNCH((wgrad_tap_kernel<DT_BF16, true>), grid, dim3(WT_NT), 0, st, p);
    else TRACKED_LAUNCH((wgrad_tap_kernel<DT_BF16, false>), grid, dim3(WT_NT), 0, st, p);
  } else if (dt == DT_F16) {
    if (pro) TRACKED_LAUNCH((wgrad_tap_kernel<DT_F16, true>), grid, dim3(WT_NT), 0, st, p);
    else TRACKED_LAUNCH((wgrad_tap_kernel<DT_F16, false>), grid, dim3(WT_NT), 0, st, p);
  } else {
    return -1;
  }
  return (int)hipGetLastError();
}

// The stem's weight-gradient slabs in the tap-reuse form (wgrad_stem_tap_kernel): slab
// [splits][64][16 taps x 16] (f32), summed by pda_wgrad_reduce as the generic kernel's. dz, y
// [Nb,H,W,64], x [Nb,H,W,16] 16-bit, k [3][64]. kb: padded rows per split (multiple of 64);
// splits = ceil(Nb (H+3)(W+3) / kb). W + 3 <= 122 (the X ring holds 4 steps + the forward halo).
int pda_wgrad_stem_tap(const void* dz, const void* y, const float* k, const void* x, float* slab,
                       int Nb, int H, int W, int kb, int splits, int dt, hipStream_t st) {
  if (kb <= 0 || (kb % 64) || H <= 0 || W <= 0 || W + 3 > 122 || !dz || !y || !k || !x || !slab)
    return -2;
  SwParams p{};
  p.dz = dz; p.y = y; p.k = k; p.x = x; p.slab = slab;
  p.Nb = Nb; p.H = H; p.W = W;
  p.Hp = H + 3; p.Wp = W + 3;
  const long long kp = (long long)Nb * p.Hp * p.Wp;
  if (kp >= (1ll << 30) || (long long)Nb * H * W * 128 >= 0x7fffffffll) return -4;
  p.Kp = (int)kp;
  p.kb = kb; p.nsteps = kb / 64; p.fhalo = 3 * p.Wp + 3;
  if ((long long)splits * kb < kp || (long long)(splits - 1) * kb >= kp) return -3;
  p.dHpWp = wt_div((uint32_t)(p.Hp * p.Wp));
  p.dWp = wt_div((uint32_t)p.Wp);
  const dim3 grid(splits);
  if (dt == DT_BF16) TRACKED_LAUNCH((wgrad_stem_tap_kernel<DT_BF16>), grid, dim3(WT_NT), 0, st, p);
  else if (dt == DT_F16) TRACKED_LAUNCH((wgrad_stem_tap_kernel<DT_F16>), grid, dim3(WT_NT), 0, st, p);
  else return -1;
  return (int)hipGetLastError();
}


}  // extern "C"
