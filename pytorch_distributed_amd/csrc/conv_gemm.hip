// Implicit-GEMM convolution for gfx950 (MI355X): forward, data-gradient and weight-gradient,
// NHWC activations, OHWI ("KRSC") weights, bf16/f16 inputs on MFMA 16x16x32 with f32 accumulation,
// or exact f32 inputs (MX_DTYPE=fp32, the reference scripts' precision) on MFMA 16x16x4 f32.
//
// Replaces cuDNN conv fwd/dgrad/wgrad of the reference stack: every
// Conv2d of ResNet (all 23 ResNet-50 shapes + the 7x7 stem) and the fc layer (as a 1x1 conv on a
// 1x1 image) go through this one kernel template:
//
//   FWD   : Y[m][n]      = sum_k A[m][k] * B[n][k]     A = im2col(X) gathered per 16-B chunk,
//                                                       B = W[Cout][R*S*Cin] (K contiguous)
//   DGRAD : dX[m][n]     = sum_k A[m][k] * B[k][n]     A = gathered dY, B = W rows (Cin contiguous)
//           stride-2 layers run as 4 parity classes (blockIdx.y) so no MFMA multiplies a
//           structural zero; each class only visits the taps that land on its pixels.
//   WGRAD : dW[n1][n2]   = sum_m A[m][n1] * B[m][n2]   A = dY, B = gathered X; split-K over m
//           (blockIdx.y) into f32 slabs, reduced deterministically by conv_wgrad_reduce.
//
// Operand tiles are staged global->VGPR->LDS (register staging: zero-fill for padding taps and
// ragged M; loads for tile t+1 are issued before the MFMAs of tile t). Two LDS tile layouts:
//   ROW  [rows][64 k] (128-B rows, 16-B chunks XOR-swizzled by row&7), fragments by ds_read_b128;
//   COL  [64 k][cols] (k-major), fragments by ds_read_b64_tr_b16 (hardware transpose read) with a
//        chunk swizzle that makes both the b128 writes and the transposed reads conflict-free.
// Block = 256 threads = 4 waves (2x2), block tile BM x BN x 64, wave tile (BM/2) x (BN/2).
// Forward epilogue stages the tile through LDS for 16-B coalesced stores and emits per-channel
// partial sum / sum-of-squares (BatchNorm statistics) per M-tile -- no extra pass over Y.
#include "common.h"

#include <cstdlib>
#include <cstring>

namespace {

constexpr int NT = 256;

// STAGES == 3 selects the LDS-DMA main loop: 512 threads (8 waves, one block per CU), operands
// copied global -> LDS by buffer_load ... lds (16 B per lane, no VGPR round trip) into a 3-slot
// ring, two k-tiles in flight across ONE barrier per k-tile (counted vmcnt, raw s_barrier).
template <int STAGES> constexpr int conv_nt() { return STAGES >= 3 ? 512 : NT; }

// one LDS-DMA piece: lane l's 16 bytes at byte voff of the buffer land at lds + 16*l (lds must be
// wave-uniform: it becomes M0). An out-of-range voff (>= the buffer's size) writes zeros.
// The builtin, not common.h dma16_asm: with it hipcc drains the HALO data gradient's pipeline
// before each tap's transposed reads (vmcnt(0)), and the asm form makes that launch 9 % faster
// alone -- but the step 0.04-0.08 ms slower (the overlapped side-stream weight gradients lose
// more than the chain gains; profiles/ab_r6.md section 15).
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char* lds, uint32_t voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16,
                                           (int)voff, 0, 0, 0);
}
template <int N> __device__ __forceinline__ void vm_wait() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

// WGRAD_BNA: WGRAD whose A operand is the BatchNorm-backward output formed while staging,
// dY = k1[c]*dz + k2[c]*y + k3[c] (a = dz, a2 = y): the stem's weight gradient is the only consumer
// of its BN-backward output, so the apply pass (and dY's write + re-read) is skipped.
//
// DGRAD_BNF: DGRAD of a 1x1 conv whose dY is a BatchNorm-backward output that is never
// materialised (the consumer-side fold of a bottleneck tail, csrc/conv_gemm.hip bn_fold_kernel):
// dY = k1*dz + k2*y + k3 with y = a2 . W^T (the conv's own forward), so
//   dX = dz . (k1 o W) + a2 . G + b,   G = W^T diag(k2) W,  b = W^T k3:
// the K loop runs over dz's Cout channels against rows [0, Cout) of B = [k1 o W ; G] and then over
// xa_c channels of the Gram operand xa (a2, formed by the BN+ReLU prologue of the forward when
// xa_sc is set) read at the dX pixel against rows [Cout, Cout + xa_c); the epilogue adds b.
//
// WGRAD_GRAM: WGRAD of a tensor against itself through its BN+ReLU, Gram = a^T a with
// a = relu(sc*y + sh) formed while staging BOTH operands (A: ak1 = sc, ak3 = sh; B: the usual
// prologue), plus the column sums s = sum_p a_p (blocks of the first N-tile accumulate their A
// chunks; per-split partials behind the slab). With them the tail fold's conv3 weight gradient
// needs no y3 read (decomposed form, see pda_wgrad_reduce):
//   dW3 = diag(k1) (dz^T a2) + diag(k2) W3 Gram(a2) + k3 s^T,   y3 = a2 W3^T.
//
// FWD_TAIL: FWD of a 1x1 stride-1 conv whose input is the PREVIOUS block's output
// a = relu(bn3(y3) + r), r = the residual (pro_mode 1) or bn_d(yd) (pro_mode 2, the downsample
// branch), formed while staging A from y3 (p.a) and r (p.pro_res) -- the tail's BN-apply pass is
// folded into its consumer: a is written once by the blocks of the first N-tile (p.pro_out, plus the
// ReLU bitmask p.pro_mask in mode 1) instead of written by an apply pass and read back by the conv.
enum Pass : int { FWD = 0, DGRAD = 1, WGRAD = 2, WGRAD_BNA = 3, DGRAD_BNF = 4, WGRAD_GRAM = 5,
                  FWD_TAIL = 6 };

template <int V> struct IC { static constexpr int value = V; };

struct ConvParams {
  const void* a;      // FWD: X [Nb,H,W,Cin]; DGRAD: dY [Nb,Ho,Wo,Cout]; WGRAD: dY
  const void* b;      // FWD: W [N][Kpad]; DGRAD: W [Cout][R][S][Cin]; WGRAD: X [Nb,H,W,Cin]
  void* out;          // FWD/DGRAD: [M][N] 16-bit (or f32 if out_f32); WGRAD: f32 slab [split][M][N]
  float* stats;       // FWD: [mtiles][2][N] partial sum / sumsq (nullable)
  const float* bias;  // FWD: [N] (nullable)
  int M, N, K;        // GEMM sizes (WGRAD: K = total rows, split by k_split)
  int Kpad;           // FWD: B row pitch
  int Nb, H, W, Cin;  // input X geometry
  int Ho, Wo, Cout;   // output Y geometry
  int R, S, stride, pad;
  int log2Cin;        // channels of the gathered tensor are a power of two (3 is padded to 8)
  int log2Cout;       // DGRAD: log2(Cout) when a power of two, else -1 (tap of a k-tile: shift)
  int out_f32;
  int relu;           // FWD epilogue relu (fc: 0)
  int k_chunk;        // WGRAD: rows per split
  int out_pitch;      // FWD/DGRAD: output row pitch (elements)
  FastDiv dHoWo, dWo, dS;   // m -> (img, y, x) decode of the *GEMM row* space; tap -> (r, s)
  int ntaps[4];       // DGRAD: taps per parity class
  int taps[4][9];     // DGRAD: tap ids (r*S+s) per parity class
  int tdy[4][9], tdx[4][9];   // DGRAD: dY offset of each class tap: (ph + pad - r) / stride, ...
  int Hc, Wc;         // DGRAD: class grid (H/stride, W/stride)
  FastDiv dHcWc, dWc;
  // fused BatchNorm-apply + ReLU prologue on the gathered activation operand (FWD: A, WGRAD: B):
  // the conv reads the PRE-BN tensor y and computes relu(y * pro_sc[c] + pro_sh[c]) while
  // staging the tile (padding stays exactly 0), so the activation is never materialised.
  const float* pro_sc;
  const float* pro_sh;
  // FWD_TAIL: the residual operand (mode 1: added as is; mode 2: with its own BN pro_sc2 / pro_sh2),
  // the materialised activation a and its ReLU bitmask (1 byte per 8 elements, mode 1; nullable)
  const void* pro_res; const float* pro_sc2; const float* pro_sh2;
  void* pro_out; uint8_t* pro_mask;
  int pro_mode;
  // DGRAD fused BatchNorm-backward epilogue (emode < 0: plain dX store)
  int emode, enq;                 // 0 relu(bn(y)), 1 relu(bn(y)+ey2), 2 relu(bn(y)+bn2(ey2)),
                                  // 3 as 1 with the ReLU mask read from emask (no residual read)
  const void* ey; const float* esc; const float* esh;
  const void* ey2; const float* esc2; const float* esh2;
  const void* eg2;                 // optional second gradient summed into dA
  const uint8_t* emask;            // mode 3: forward ReLU bitmask of a (1 byte per 8 elements)
  float* epart;                    // [ncls*tiles_m][enq][N] partial sums
  const void* a2;                  // WGRAD_BNA: y (the BN input) beside a = dz
  const float* ak1; const float* ak2; const float* ak3;   // WGRAD_BNA: per-Cout coefficients
  // DGRAD_BNF: the Gram operand (xa_c channels at the dX pixel; BN+ReLU applied when xa_sc is set)
  // and the epilogue bias b[N]
  const void* xa; const float* xa_sc; const float* xa_sh; const float* dbias;
  int xa_c;
  int rev;   // walk each XCD's tile chunk from its end (xcd_remap_rev; PDA_REVERSE experiments)
  // FWD BatchNorm statistics (stats != nullptr) are per-M-tile SHIFTED partials
  // stats[tile][3][N] = (sum(y - s), sum((y - s)^2), s), s = the tile's first row (no f32
  // cancellation when |mean| >> std); bn.hip bn_fwd_stats combines and finalizes them.
};

// Scalar-f32 pair FMA for the operand prologue, which runs between MFMAs: there a packed
// v_pk_fma_f32 costs far more issue time than two scalar v_fma_f32 (MI355X_MICROARCH.md, cycle
// constants). This file is built with -fno-slp-vectorize so the compiler does not re-pack them.
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) {
  return f32x2{__builtin_fmaf(a.x, b.x, c.x), __builtin_fmaf(a.y, b.y, c.y)};
}

// ---------------------------------------------------------------- LDS addressing
// ROW tile: BR rows x 64 k (128 B per row).
__device__ __forceinline__ int row_addr(int row, int chunk) {
  return row * 128 + ((chunk ^ (row & 7)) << 4);
}
// COL tile: 64 k-rows x BC cols.
template <int BC>
__device__ __forceinline__ int col_swz(int krow) {
  // BC >= 128: only (address mod 256 B) picks the bank, so the 128-column pattern also makes the
  // 256-column tile (512-B rows) conflict-free for the b128 writes and the transposed reads
  if constexpr (BC >= 128) return ((krow & 3) << 1) | (((krow >> 3) & 1) << 3);
  else return (((krow >> 1) & 1) << 1) | (((krow >> 3) & 1) << 2);
}
template <int BC>
__device__ __forceinline__ int col_addr(int krow, int chunk) {
  return krow * (BC * 2) + ((chunk ^ col_swz<BC>(krow)) << 4);
}

// fragment loads -------------------------------------------------------------------
// ROW tile, operand rows [rb, rb+16), k-step s (32 k): lane holds row rb+(l&15), k 8*(l>>4)..+7
__device__ __forceinline__ s16x8 frag_row(const char* lds, int rb, int s, int lane) {
  const int row = rb + (lane & 15);
  const int chunk = s * 4 + (lane >> 4);
  return *reinterpret_cast<const s16x8*>(lds + row_addr(row, chunk));
}
// COL tile, operand cols [cb, cb+16), k-step s: lane holds col cb+(l&15), k 8*(l>>4)..+7
template <int BC>
__device__ __forceinline__ s16x8 frag_col(const char* lds, int cb, int s, int lane) {
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int chunk = (cb >> 3) + (p >> 1);
  const int k0 = s * 32 + 8 * g + q;
  const int a0 = col_addr<BC>(k0, chunk) + ((p & 1) << 3);
  const int a1 = col_addr<BC>(k0 + 4, chunk) + ((p & 1) << 3);
  s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + a0));
  s16x4 v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, lds + a1));
  s16x8 r;
  r[0] = v0[0]; r[1] = v0[1]; r[2] = v0[2]; r[3] = v0[3];
  r[4] = v1[0]; r[5] = v1[1]; r[6] = v1[2]; r[7] = v1[3];
  return r;
}

// COL tile of f32 (exact-fp32 path): 32 k-rows x BC cols of 4 B, 16-B chunks XOR-swizzled by
// 4 * ((krow >> 2) & 3) so the four k-groups of a fragment read land in disjoint bank quarters.
template <int BC>
__device__ __forceinline__ int col_addr_f32(int krow, int chunk) {
  return krow * (BC * 4) + ((chunk ^ (((krow >> 2) & 3) << 2)) << 4);
}
// lane holds col cb+(l&15), k = 16*s + 4*(l>>4) + 0..3 (the k order of frag_row on an f32 ROW tile)
template <int BC>
__device__ __forceinline__ f32x4 frag_col_f32(const char* lds, int cb, int s, int lane) {
  const int g = lane >> 4, col = cb + (lane & 15);
  f32x4 r;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int krow = s * 16 + 4 * g + j;
    r[j] = *reinterpret_cast<const float*>(lds + col_addr_f32<BC>(krow, col >> 2) + ((col & 3) << 2));
  }
  return r;
}

// ================================================================= kernel
// STAGES = 2: double-buffered LDS, one barrier per k-tile (deep-K layers).
// STAGES = 1: single LDS buffer (half the LDS -> one more resident block per CU) for the many
//             shallow-K layers of ResNet (K = 64..128: nk <= 2), where the per-block
//             load -> MFMA -> store chain is latency-bound and concurrency matters more.
// Resident blocks per CU the register allocation must allow (one wave per SIMD per block): the
// 16-bit 64x64 and single-stage 128x64 / 64x128 tiles are held to 5 / 4 (<= 96 / 128 VGPRs) --
// their fused epilogues would otherwise push them a few registers over and cost a wave per SIMD.
// 256-wide tiles (single-stage only; wave tile 128x64 / 64x128: a quarter less LDS traffic per
// MFMA) need ~250 registers and 64 KiB of LDS: two blocks per CU.
template <int DT, int BM, int BN, int STAGES>
constexpr int conv_min_blocks() {
  if (STAGES >= 3) return 2;   // one 512-thread block per CU = two waves per SIMD
  if (DT == DT_F32S) return BM * BN <= 64 * 64 ? 4 : 2;   // hi + lo tiles: twice the LDS
  if (DT != DT_F32 && BM * BN <= 64 * 64) return 5;
  if (DT != DT_F32 && STAGES == 1 && BM * BN <= 128 * 64) return 4;
  if (BM > 128) return 2;   // 256-row register tiles (8 A chunks per thread): 3 blocks spill
  return (STAGES == 1 && BM * BN <= 128 * 128) ? 3 : 2;
}

template <int PASS_T, int DT, int BM, int BN, int STAGES>
// WGRAD_BNA holds the fixed column chunk's 24 BN coefficients and the y chunks: 3 blocks per CU
// (the 16-bit WGRAD budget of 4 spilled 15 VGPRs); its 256-column tile (the stem's whole N: dz and
// y staged and transformed once instead of once per 128-column tile) needs 246: 2 blocks per CU
// (the 128x128 WGRAD_BNA tile of the bottleneck conv3 fold: 2 blocks, 3 spilled 89 VGPRs)
// FWD_TAIL holds the residual chunks and both branches' BN coefficients across the MFMAs: the
// 128x64 tile at 3 blocks per CU, 128x128 at 2 (the plain FWD budgets spill 43 / 50 VGPRs)
__global__ __launch_bounds__(conv_nt<STAGES>(), (PASS_T == WGRAD_BNA || PASS_T == WGRAD_GRAM ? (BN >= 256 || BM * BN >= 128 * 128 ? 2 : 3) : PASS_T == FWD_TAIL ? (BM * BN >= 128 * 128 ? 2 : 3) : conv_min_blocks<DT, BM, BN, STAGES>())) void conv_gemm_kernel(ConvParams p_arg) {
  constexpr int PASS = PASS_T == WGRAD_BNA || PASS_T == WGRAD_GRAM ? WGRAD
                       : PASS_T == DGRAD_BNF ? DGRAD : PASS_T == FWD_TAIL ? FWD : PASS_T;
  constexpr bool TAILP = PASS_T == FWD_TAIL;   // tail-apply prologue (a = relu(bn3(y3) + r))
  constexpr bool GRAM = PASS_T == WGRAD_GRAM;   // A = relu(ak1*a + ak3); no second tensor
  constexpr bool ABN = PASS_T == WGRAD_BNA || GRAM;
  constexpr bool BNF = PASS_T == DGRAD_BNF;
  constexpr bool DMA = STAGES >= 3;
  // STAGES == 4 (HALO): tap reuse for 3x3 stride-1 FWD / DGRAD -- see the HALO main loop
  constexpr bool HALO = STAGES == 4;
  constexpr int NTH = conv_nt<STAGES>();
  // wave grid: 2x2 (256 threads); DMA: 4x2 or 2x4 so the wave tile stays square-ish
  constexpr int WM = DMA ? (BM >= BN ? 4 : 2) : 2;
  constexpr int WN = (NTH / 64) / WM;
  static_assert(!DMA || ((DT == DT_BF16 || DT == DT_F16) && !ABN), "LDS-DMA: 16-bit");
  static_assert(!ABN || DT == DT_BF16 || DT == DT_F16, "WGRAD_BNA: 16-bit operands");
  static_assert(!BNF || ((DT == DT_BF16 || DT == DT_F16) && !DMA), "DGRAD_BNF: 16-bit, register-staged");
  static_assert(!TAILP || ((DT == DT_BF16 || DT == DT_F16) && STAGES == 1), "FWD_TAIL: 16-bit, single-stage");
  // DGRAD / WGRAD read the parameters in place in the kernarg segment (constant address space):
  // binding a reference to the by-value argument makes the compiler copy the whole ~1 KB block to
  // scratch once a member array is indexed dynamically (DGRAD tap tables), and costs WGRAD spills.
  // FWD keeps the plain argument -- read in place, the compiler re-issues scalar kernarg loads
  // (with their waits) per epilogue row instead of holding the fields in SGPRs.
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) ConvParams KParams;
  auto&& p = [&]() -> decltype(auto) {
    if constexpr (PASS != FWD) return *(KParams*)__builtin_amdgcn_kernarg_segment_ptr();
    else return (p_arg);
  }();
#else   // host pass of the template (never executed): the plain argument
  const ConvParams& p = p_arg;
#endif
  // A tile: FWD/DGRAD ROW [BM][64]; WGRAD COL [64][BM]. B tile: FWD ROW [BN][64]; else COL [64][BN]
  // element geometry: 16-bit operands move 8 elements per 16-B chunk and 64 k per 128-B tile row;
  // the exact-f32 path (DT_F32, MFMA 16x16x4 f32) moves 4 per chunk and 32 k per row; the split
  // path (DT_F32S) reads f32 tensors (two 16-B loads per 8-element chunk) and stages bf16 hi and
  // lo tiles in the 16-bit LDS layout (the lo images AB_BYTES behind the hi images)
  constexpr bool F32 = DT == DT_F32;
  constexpr bool SPLIT = DT == DT_F32S;
  constexpr bool O32 = F32 || SPLIT;     // f32 tensors in memory (operands and C tile)
  constexpr int MDT = SPLIT ? DT_BF16 : DT;   // MFMA / pack element type of the 16-bit paths
  constexpr int LES = F32 ? 4 : 2;       // operand element bytes in LDS
  constexpr int ES = O32 ? 4 : 2;        // element bytes in global memory and in the C tile
  constexpr int EPC = 16 / LES;          // operand elements per 16-B LDS chunk
  constexpr int EPO = 16 / ES;           // C-tile elements per 16-B chunk (epilogue)
  // k per tile: one 128-B row; the 256x256 LDS-DMA tile (weight gradient: both images k-major)
  // takes 32 k per tile so that four ring slots (128 KiB) keep three tiles in flight
  constexpr bool BK32 = DMA && !HALO && BM * BN >= 256 * 256;
  constexpr int BKE = BK32 ? 32 : 128 / LES;
  static_assert(!BK32 || PASS == WGRAD, "the 32-k tile has k-major (COL) images only");
  constexpr int A_BYTES = BM * BKE * LES, B_BYTES = BN * BKE * LES;
  constexpr int AB_BYTES = A_BYTES + B_BYTES;
  constexpr int STAGE = SPLIT ? 2 * AB_BYTES : AB_BYTES;
  // epilogue partial-sum reduction [3][RG][BN] f32
  constexpr int RED_BYTES = 3 * NTH * 8 * 4;
  // staged C tile of the epilogue; f32 stages it in two row halves (one per wave row), so the
  // epilogue needs no more LDS than the main loop and f32 tiles keep 3 resident blocks per CU
  constexpr int NH = O32 ? 2 : 1;
  constexpr int C_BYTES = BM / NH * BN * ES;
  // HALO: two input-slab slots of BM + 128 rows (any W <= 63: BM + 2W + 2 rows), three weight-tile
  // slots and one zero row (the fragment source of a tap that falls outside the image; a masked
  // lane's broadcast read of it shares a bank quad with an unmasked lane: the ~22 % LDS conflicts
  // of these launches -- a per-lane zero address removes them but costs 34 VGPRs and spills,
  // profiles/ab_r6.md section 10)
  constexpr int SLAB_ROWS = BM + 128, SLAB_BYTES = SLAB_ROWS * 128;
  constexpr int ZOFF = 2 * SLAB_BYTES + 3 * B_BYTES;
  // LDS-DMA ring slots: 4 when they fit in 144 KiB (three tiles in flight), else 3
  // (CONV_WGRAD_DMA_SLOTS, a build-time A/B knob: ring depth of the weight-gradient DMA tiles,
  // whose LDS footprint decides whether a main-stream block fits beside one on its CU)
#ifndef CONV_WGRAD_DMA_SLOTS
#define CONV_WGRAD_DMA_SLOTS 0
#endif
  constexpr int NSLOT = DMA && !HALO
      ? (PASS == WGRAD && CONV_WGRAD_DMA_SLOTS > 0 ? CONV_WGRAD_DMA_SLOTS
                                                   : (4 * STAGE <= 144 * 1024 ? 4 : 3))
      : STAGES;
  static_assert(!DMA || HALO || NSLOT >= 2, "DMA ring");
  constexpr int RING = HALO ? ZOFF + 128 : NSLOT * STAGE;
  constexpr int LDS_0 = RING > RED_BYTES ? RING : RED_BYTES;
  constexpr int LDS_BYTES = LDS_0 > C_BYTES ? LDS_0 : C_BYTES;
  static_assert(BN <= NTH, "stats reduction: one thread per column");
  static_assert(C_BYTES <= LDS_BYTES, "C tile must fit in the staging buffers");
  static_assert(RED_BYTES <= LDS_BYTES, "stats reduction must fit");
  __shared__ __attribute__((aligned(16))) char smem[LDS_BYTES];

  constexpr bool A_ROW = (PASS != WGRAD);
  constexpr bool B_ROW = (PASS == FWD);
  constexpr int AR = BM / 32, BR = BN / 32;  // 16-B chunks per thread per tile

  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wid / WN, wc = wid % WN;
  const int tiles_n = (p.N + BN - 1) / BN;
  const int tiles_m = (p.M + BM - 1) / BM;
  const int ntile = tiles_m * tiles_n;
  const int t = (int)(p.rev ? xcd_remap_rev(blockIdx.x, ntile) : xcd_remap(blockIdx.x, ntile));
  const int tm = t / tiles_n, tn = t - tm * tiles_n;
  const int m0 = tm * BM, n0 = tn * BN;
  const int split = blockIdx.y;  // WGRAD: K split; DGRAD: parity class

  // ---- K range --------------------------------------------------------------------
  int kbeg = 0, kend = p.K;
  int cls_ph = 0, cls_pw = 0, ntap = 0;
  if constexpr (PASS == WGRAD) {
    kbeg = split * p.k_chunk;
    kend = min(p.K, kbeg + p.k_chunk);
  } else if constexpr (PASS == DGRAD) {
    cls_ph = split >> 1;
    cls_pw = split & 1;
    ntap = p.ntaps[split];
    kend = ntap * p.Cout;
    if (BNF && ntap > 0) kend += p.xa_c;   // the Gram operand's k-tiles (landing classes only)
  }
  const int nk = (kend - kbeg + BKE - 1) / BKE;

  // ---- per-thread loader precompute -------------------------------------------------
  // Operands are read with buffer loads (32-bit byte offsets, hardware range check): a padding
  // tap / ragged row / ragged column gets offset OOB and the load returns zeros -- no branch
  // around the load, no 64-bit address math. Everything that does not change along K is hoisted
  // here, so a k-tile costs ~1-3 VALU per 16-byte chunk (+ one tap decode per thread).
  // A (ROW: FWD gather from X, DGRAD gather from dY): rows tid/8 + 32*i, chunk tid&7
  constexpr uint32_t OOB = 0x80000000u;
  int a_base[AR];           // byte offset of the row's tap-(0,0) pixel (FWD/DGRAD), may be < 0
  uint32_t xa_base[BNF ? AR : 1];   // DGRAD_BNF: byte offset of the row's dX pixel in xa
  uint64_t a_mask[AR];      // bit t: tap t (FWD, R*S <= 64) / class tap t (DGRAD) is inside the image
  uint32_t a_off[AR];       // WGRAD: byte offset of (krow, col) at k0 = kbeg
  int a_krow[AR];
  if constexpr (A_ROW) {
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      const int m = m0 + (tid >> 3) + 32 * i;
      const bool okm = m < p.M;
      const uint32_t mm = okm ? m : 0;
      uint64_t msk = 0;
      if constexpr (PASS == FWD) {
        const uint32_t img = fdiv(mm, p.dHoWo), rem = mm - img * p.dHoWo.d;
        const uint32_t yo = fdiv(rem, p.dWo), xo = rem - yo * p.dWo.d;
        const int y0 = (int)yo * p.stride - p.pad, x0 = (int)xo * p.stride - p.pad;
        a_base[i] = (((int)img * p.H + y0) * p.W + x0) * p.Cin * ES;
        for (int r = 0, t = 0; r < p.R; ++r) {
          const bool yok = (unsigned)(y0 + r) < (unsigned)p.H;
          for (int q = 0; q < p.S; ++q, ++t)
            if (yok && (unsigned)(x0 + q) < (unsigned)p.W) msk |= 1ull << t;
        }
      } else {  // DGRAD: class-grid pixel (yi, xi); tap t of the class reads dY[yi + dy_t][xi + dx_t]
        const uint32_t img = fdiv(mm, p.dHcWc), rem = mm - img * p.dHcWc.d;
        const uint32_t yi = fdiv(rem, p.dWc), xi = rem - yi * p.dWc.d;
        a_base[i] = (((int)img * p.Ho + (int)yi) * p.Wo + (int)xi) * p.Cout * ES;
        for (int t = 0; t < ntap; ++t) {
          if ((unsigned)((int)yi + p.tdy[split][t]) < (unsigned)p.Ho &&
              (unsigned)((int)xi + p.tdx[split][t]) < (unsigned)p.Wo)
            msk |= 1ull << t;
        }
        if constexpr (BNF) {
          const uint32_t h = yi * p.stride + cls_ph, w = xi * p.stride + cls_pw;
          xa_base[i] = ((img * p.H + h) * p.W + w) * (uint32_t)p.xa_c * (uint32_t)ES;
        }
      }
      a_mask[i] = okm ? msk : 0ull;
    }
  } else {
    constexpr int CPR = BM / EPC, RPI = NT / CPR;
    const int col = m0 + (tid % CPR) * EPC;
#pragma unroll
    for (int i = 0; i < AR; ++i) {
      a_krow[i] = tid / CPR + RPI * i;
      a_off[i] = col < p.M ? (uint32_t)((kbeg + a_krow[i]) * p.Cout + col) * (uint32_t)ES : OOB;
    }
  }
  // WGRAD_BNA: the thread's A column chunk (8 output channels) is fixed: its coefficients once
  f32x2 bk1[ABN ? 4 : 1], bk2[ABN ? 4 : 1], bk3[ABN ? 4 : 1];
  if constexpr (ABN) {
    constexpr int CPR = BM / EPC;
    const int col = m0 + (tid % CPR) * EPC;
    const int cs = col < p.M ? col : 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bk1[k] = *reinterpret_cast<const f32x2*>(p.ak1 + cs + 2 * k);
      if constexpr (!GRAM) bk2[k] = *reinterpret_cast<const f32x2*>(p.ak2 + cs + 2 * k);
      bk3[k] = *reinterpret_cast<const f32x2*>(p.ak3 + cs + 2 * k);
    }
  }
  // WGRAD_GRAM: column sums of the thread's A chunk (the 8 channels of its column), first N-tile
  f32x2 gsum[GRAM ? 4 : 1];
#pragma unroll
  for (int k = 0; k < (GRAM ? 4 : 1); ++k) gsum[k] = f32x2{0.f, 0.f};
  const bool gcol = GRAM && tn == 0;
  // WGRAD_GRAM diagonal tile (tm == tn, square tile): the B image IS the A image (same tensor, same
  // rows, same channels, same BN+ReLU) -- loaded, transformed and stored once, read twice
  const bool gsame = GRAM && BM == BN && tm == tn;
  // B
  uint32_t b_off[BR];
  if constexpr (PASS == FWD) {
#pragma unroll
    for (int i = 0; i < BR; ++i) {
      const int n = n0 + (tid >> 3) + 32 * i;
      b_off[i] = n < p.N ? (uint32_t)(n * p.Kpad + (tid & 7) * EPC) * (uint32_t)ES : OOB;
    }
  } else if constexpr (PASS == DGRAD) {
    constexpr int CPR = BN / EPC, RPI = NT / CPR;
    const int col = n0 + (tid % CPR) * EPC;
#pragma unroll
    for (int i = 0; i < BR; ++i)
      b_off[i] = col < p.N ? (uint32_t)((tid / CPR + RPI * i) * p.R * p.S * p.Cin + col) * (uint32_t)ES : OOB;
  }
  // WGRAD B gather: fixed column chunk per thread -> (tap, c)
  int wb_r = 0, wb_s = 0, wb_c = 0;
  bool wb_colok = true;
  const bool wb_direct = PASS == WGRAD && p.R == 1 && p.S == 1 && p.stride == 1 && p.pad == 0;
  if constexpr (PASS == WGRAD) {
    constexpr int CPR = BN / EPC;
    const int col = n0 + (tid % CPR) * EPC;
    wb_colok = col < p.N;
    const int tap = col >> p.log2Cin;
    wb_c = col & ((1 << p.log2Cin) - 1);
    wb_r = (int)fdiv(tap, p.dS);
    wb_s = tap - wb_r * p.S;
    wb_colok = wb_colok && (tap < p.R * p.S);
  }

  // buffer resources (wave-uniform: built from kernel arguments only)
  uint32_t a_bytes, b_bytes;
  if constexpr (PASS == FWD) {
    a_bytes = (uint32_t)p.Nb * p.H * p.W * p.Cin * (uint32_t)ES;
    b_bytes = (uint32_t)p.N * p.Kpad * (uint32_t)ES;
  } else if constexpr (PASS == DGRAD) {
    a_bytes = (uint32_t)p.Nb * p.Ho * p.Wo * p.Cout * (uint32_t)ES;
    b_bytes = (uint32_t)(p.Cout + (BNF ? p.xa_c : 0)) * p.R * p.S * p.Cin * (uint32_t)ES;
  } else {
    a_bytes = (uint32_t)p.K * p.Cout * (uint32_t)ES;
    b_bytes = (uint32_t)p.Nb * p.H * p.W * p.Cin * (uint32_t)ES;
  }
  const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.a), (short)0,
                                                                         (int)a_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rsb = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p.b), (short)0,
                                                                         (int)b_bytes, 0x00020000);
  auto bld = [&](const __amdgpu_buffer_rsrc_t& r, uint32_t off) __attribute__((always_inline)) -> i32x4 {
    return __builtin_bit_cast(i32x4, __builtin_amdgcn_raw_buffer_load_b128(r, (int)off, 0, 0));
  };
  // WGRAD_BNA: y beside dz (same geometry), its chunks and the chunks' validity (padding rows must
  // stay 0, not k3)
  const __amdgpu_buffer_rsrc_t rsa2 = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(ABN ? p.a2 : p.a), (short)0, (int)a_bytes, 0x00020000);
  i32x4 ray[ABN ? AR : 1];
  bool av[ABN ? AR : 1];
  // DGRAD_BNF: the Gram operand (the dX-resolution tensor, xa_c channels)
  const __amdgpu_buffer_rsrc_t rsx = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(BNF ? p.xa : p.a), (short)0,
      BNF ? (int)((uint32_t)p.Nb * p.H * p.W * p.xa_c * (uint32_t)ES) : (int)a_bytes, 0x00020000);
  bool xt = false;   // DGRAD_BNF: the tile in the staging registers is a Gram-operand tile
  // FWD_TAIL: the residual (same geometry as A), its staged chunks, the staged tile's channel base
  const __amdgpu_buffer_rsrc_t rsr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<void*>(TAILP ? p.pro_res : p.a), (short)0, (int)a_bytes, 0x00020000);
  i32x4 rres[TAILP ? AR : 1];
  int st_c = 0, st_c_w = 0;     // channel base of the loaded / of the staged k-tile
  uint32_t tail_bits = 0;       // ReLU bits of the staged chunks (byte i: chunk i)
  const bool tail_wr = TAILP && tn == 0;   // the first N-tile's blocks write a (each A chunk once)

  i32x4 ra[AR], rb[BR];
  i32x4 ra2[SPLIT ? AR : 1], rb2[SPLIT ? BR : 1];   // DT_F32S: elements 4..7 of each chunk
  auto lda = [&](int i, uint32_t off) __attribute__((always_inline)) {
    ra[i] = bld(rsa, off);
    if constexpr (SPLIT) ra2[i] = bld(rsa, off + 16u);   // OOB + 16 stays out of range
  };
  auto ldb = [&](int i, uint32_t off) __attribute__((always_inline)) {
    rb[i] = bld(rsb, off);
    if constexpr (SPLIT) rb2[i] = bld(rsb, off + 16u);
  };
  // prologue state: per-chunk validity (padding must stay 0) and the chunk's 8 channel coeffs
  const bool pro = (PASS == FWD || PASS == WGRAD) && (TAILP || p.pro_sc != nullptr);
  const bool xpro = BNF && p.xa_sc != nullptr;   // DGRAD_BNF: BN+ReLU on the Gram operand
  bool pv[PASS == WGRAD ? BR : AR];
  f32x2 psc[4], psh[4];
  f32x2 psc2[TAILP ? 4 : 1], psh2[TAILP ? 4 : 1];
  auto pro_coeffs_of = [&](const float* sc, const float* sh, int c) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < EPC / 2; ++k) {
      psc[k] = *reinterpret_cast<const f32x2*>(sc + c + 2 * k);
      psh[k] = *reinterpret_cast<const f32x2*>(sh + c + 2 * k);
      if constexpr (TAILP) {
        if (p.pro_mode == 2) {
          psc2[k] = *reinterpret_cast<const f32x2*>(p.pro_sc2 + c + 2 * k);
          psh2[k] = *reinterpret_cast<const f32x2*>(p.pro_sh2 + c + 2 * k);
        }
      }
    }
  };
  auto pro_coeffs = [&](int c) __attribute__((always_inline)) { pro_coeffs_of(p.pro_sc, p.pro_sh, c); };
  if (PASS == WGRAD && pro) pro_coeffs(wb_colok ? wb_c : 0);
  // relu on the packed 16-bit result: bf16/f16 are sign-magnitude, so a signed 16-bit max with 0
  // zeroes exactly the negative values (and -0) -- one v_pk_max_i16 per pair
  typedef short s16x2 __attribute__((ext_vector_type(2)));
  auto pro_apply = [&](i32x4& v) __attribute__((always_inline)) {
    if constexpr (F32) {   // one f32 element per dword
#pragma unroll
      for (int k = 0; k < 4; ++k)
        v[k] = __float_as_int(fmaxf(__builtin_fmaf(__int_as_float(v[k]), psc[k >> 1][k & 1],
                                                   psh[k >> 1][k & 1]), 0.f));
    } else if constexpr (!SPLIT) {   // (DT_F32S: pro_apply2)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const f32x2 u = unpack2<DT>((uint32_t)v[k]);
        const f32x2 f = fma2(u, psc[k], psh[k]);
        const s16x2 h = __builtin_bit_cast(s16x2, pack2<DT>(f));
        v[k] = __builtin_bit_cast(int, __builtin_elementwise_max(h, (s16x2){0, 0}));
      }
    }
  };

  // FWD_TAIL: a = relu(bn3(y3) + r) on the chunk (the same fma chain as the apply pass,
  // common.h tail_act2, so the written activation is bit-identical to it); returns the ReLU bits
  auto tail_apply = [&](i32x4& v, const i32x4& r) __attribute__((always_inline)) -> uint32_t {
    uint32_t bits = 0;
    if constexpr (TAILP) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        f32x2 a = tail_pre2(unpack2<DT>((uint32_t)v[k]), psc[k], psh[k],
                            unpack2<DT>((uint32_t)r[k]), psc2[k], psh2[k], p.pro_mode);
        a = f32x2{fmaxf(a.x, 0.f), fmaxf(a.y, 0.f)};
        v[k] = (int)pack2<DT>(a);
        bits |= (a.x > 0.f ? 1u : 0u) << (2 * k);
        bits |= (a.y > 0.f ? 1u : 0u) << (2 * k + 1);
      }
    }
    return bits;
  };

  // DT_F32S: BN+ReLU on the chunk's 8 f32 values (v0: channels 0-3, v1: 4-7)
  auto pro_apply2 = [&](i32x4& v0, i32x4& v1) __attribute__((always_inline)) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v0[k] = __float_as_int(fmaxf(__builtin_fmaf(__int_as_float(v0[k]), psc[k >> 1][k & 1],
                                                  psh[k >> 1][k & 1]), 0.f));
      v1[k] = __float_as_int(fmaxf(__builtin_fmaf(__int_as_float(v1[k]), psc[2 + (k >> 1)][k & 1],
                                                  psh[2 + (k >> 1)][k & 1]), 0.f));
    }
  };
  // DT_F32S: 8 f32 -> bf16 hi chunk at base+addr and bf16 lo = bf16(x - hi) chunk AB_BYTES behind
  auto split_put = [&](char* base, int addr, const i32x4& v0, const i32x4& v1)
      __attribute__((always_inline)) {
    i32x4 hi, lo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const i32x4& v = k < 2 ? v0 : v1;
      const f32x2 f = f32x2{__int_as_float(v[2 * (k & 1)]), __int_as_float(v[2 * (k & 1) + 1])};
      const uint32_t h = pack2<DT_BF16>(f);
      hi[k] = (int)h;
      lo[k] = (int)pack2<DT_BF16>(f - unpack2<DT_BF16>(h));
    }
    *reinterpret_cast<i32x4*>(base + addr) = hi;
    *reinterpret_cast<i32x4*>(base + AB_BYTES + addr) = lo;
  };

  auto load_tile = [&](int kt) __attribute__((always_inline)) {
    const int k0 = kbeg + kt * BKE;
    // ---------------- A
    if constexpr (PASS == FWD) {
      if (p.Cin >= BKE) {
        // the k-tile lies in ONE tap (Cin is a power of two >= 64): tap, (r, s) and the tap's
        // pixel offset are wave-uniform scalar math; per lane only the chunk's channel offset
        const int tap = k0 >> p.log2Cin;
        const int c0 = k0 & ((1 << p.log2Cin) - 1);
        const int r = (int)fdiv(tap, p.dS), q = tap - r * p.S;
        const int toff = ((r * p.W + q) * p.Cin + c0 + (tid & 7) * EPC) * ES;
        const uint32_t word = tap >> 5, bit = tap & 31;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const uint32_t mw = word ? (uint32_t)(a_mask[i] >> 32) : (uint32_t)a_mask[i];
          const bool ok = (mw >> bit) & 1u;
          lda(i, ok ? (uint32_t)(a_base[i] + toff) : OOB);
          if constexpr (TAILP) rres[i] = bld(rsr, ok ? (uint32_t)(a_base[i] + toff) : OOB);
          pv[i] = ok;
        }
        if constexpr (TAILP) st_c = c0;
        if (pro) pro_coeffs(c0 + (tid & 7) * EPC);
      } else {   // Cin < 64 (the space-to-depth stem): taps change inside the k-tile
        const int k = k0 + (tid & 7) * EPC;
        const int tap = k >> p.log2Cin;
        const int c = k & ((1 << p.log2Cin) - 1);
        const int r = (int)fdiv(tap, p.dS), q = tap - r * p.S;
        const int toff = ((r * p.W + q) * p.Cin + c) * ES;
        const bool tap_ok = tap < p.R * p.S;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const bool ok = tap_ok && ((a_mask[i] >> (tap & 63)) & 1ull);
          lda(i, ok ? (uint32_t)(a_base[i] + toff) : OOB);
          pv[i] = ok;
        }
        if (pro) pro_coeffs(c);
      }
    } else if constexpr (PASS == DGRAD) {
      if (BNF && k0 >= ntap * p.Cout) {   // Gram-operand tile: xa at the dX pixel
        const int c = k0 - ntap * p.Cout + (tid & 7) * EPC;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const bool ok = ((uint32_t)a_mask[i]) & 1u;   // valid row (1x1: its tap lands)
          ra[i] = bld(rsx, ok ? xa_base[i] + (uint32_t)(c * ES) : OOB);
          pv[i] = ok;
        }
        if (xpro) pro_coeffs_of(p.xa_sc, p.xa_sh, c);
        xt = true;
      } else {
        // tile lies in one tap (Cout % 64 == 0); scalar shift instead of a scalar division
        const int ti = p.log2Cout >= 0 ? k0 >> p.log2Cout : k0 / p.Cout;
        const int c = k0 - ti * p.Cout + (tid & 7) * EPC;
        const int tsel = ti < 9 ? ti : 0;
        const int toff = ((p.tdy[split][tsel] * p.Wo + p.tdx[split][tsel]) * p.Cout + c) * ES;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
          const bool ok = ((uint32_t)a_mask[i] >> ti) & 1u;
          lda(i, ok ? (uint32_t)(a_base[i] + toff) : OOB);
        }
        if constexpr (BNF) xt = false;
      }
    } else {  // WGRAD A: dY rows m (k), cols n1 (COL tile [64][BM])
      const uint32_t koff = (uint32_t)(kt * BKE * p.Cout) * (uint32_t)ES;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        const bool ok = k0 + a_krow[i] < kend;
        lda(i, ok ? a_off[i] + koff : OOB);
        if constexpr (ABN) {
          if constexpr (!GRAM) ray[i] = bld(rsa2, ok ? a_off[i] + koff : OOB);
          av[i] = ok && a_off[i] != OOB;
        }
      }
    }
    // ---------------- B
    if constexpr (PASS == FWD) {
#pragma unroll
      for (int i = 0; i < BR; ++i) ldb(i, b_off[i] + (uint32_t)k0 * (uint32_t)ES);
    } else if constexpr (PASS == DGRAD) {
      const int ti = p.log2Cout >= 0 ? k0 >> p.log2Cout : k0 / p.Cout;
      const int tap = p.taps[split][ti < 9 ? ti : 0];
      uint32_t uoff = (uint32_t)(((k0 - ti * p.Cout) * p.R * p.S + tap) * p.Cin) * (uint32_t)ES;
      if (BNF && k0 >= ntap * p.Cout) uoff = (uint32_t)(k0 * p.Cin) * (uint32_t)ES;   // rows of G (1x1)
#pragma unroll
      for (int i = 0; i < BR; ++i) ldb(i, b_off[i] + uoff);
    } else if (wb_direct) {  // WGRAD B, 1x1 stride-1 conv: X rows ARE the GEMM rows
      constexpr int CPR = BN / EPC, RPI = NT / CPR;
      if (gsame) return;
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const int m = k0 + tid / CPR + RPI * i;
        const bool ok = wb_colok && m < kend;
        ldb(i, ok ? (uint32_t)(m * p.Cin + wb_c) * (uint32_t)ES : OOB);
        pv[i] = ok;
      }
    } else {  // WGRAD B: gathered X rows m, cols (tap, c)
      constexpr int CPR = BN / EPC, RPI = NT / CPR;
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const int krow = tid / CPR + RPI * i;
        const int m = k0 + krow;
        bool ok = wb_colok && m < kend;
        const uint32_t mm = ok ? m : 0;
        const uint32_t img = fdiv(mm, p.dHoWo), rem = mm - img * p.dHoWo.d;
        const uint32_t yo = fdiv(rem, p.dWo), xo = rem - yo * p.dWo.d;
        const int y = (int)yo * p.stride - p.pad + wb_r, x = (int)xo * p.stride - p.pad + wb_s;
        ok = ok && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
        const int off = ((((int)img * p.H + y) * p.W + x) * p.Cin + wb_c) * ES;
        ldb(i, ok ? (uint32_t)off : OOB);
        if constexpr (PASS == WGRAD) pv[i] = ok;
      }
    }
  };

  auto store_tile = [&](int buf) __attribute__((always_inline)) {
    char* sa = smem + buf * STAGE;
    char* sb = sa + A_BYTES;
    if constexpr (A_ROW) {
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        if constexpr (TAILP) {
          if (i == 0) { st_c_w = st_c; tail_bits = 0; }
          if (pv[i]) tail_bits |= tail_apply(ra[i], rres[i]) << (8 * i);
        } else if constexpr (PASS == FWD) {
          if constexpr (SPLIT) {
            if (pro && pv[i]) pro_apply2(ra[i], ra2[i]);
          } else {
            if (pro && pv[i]) pro_apply(ra[i]);
          }
        }
        if constexpr (BNF) {
          if (xt && xpro && pv[i]) pro_apply(ra[i]);
        }
        const int addr = row_addr((tid >> 3) + 32 * i, tid & 7);
        if constexpr (SPLIT) split_put(sa, addr, ra[i], ra2[i]);
        else *reinterpret_cast<i32x4*>(sa + addr) = ra[i];
      }
    } else {
      constexpr int CPR = BM / EPC, RPI = NT / CPR;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        if constexpr (GRAM) {   // a = relu(sc*y + sh) on the valid chunks (padding stays 0)
          if (av[i]) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const f32x2 u = unpack2<DT>((uint32_t)ra[i][k]);
              const s16x2 h = __builtin_bit_cast(s16x2, pack2<DT>(fma2(u, bk1[k], bk3[k])));
              ra[i][k] = __builtin_bit_cast(int, __builtin_elementwise_max(h, (s16x2){0, 0}));
              if (gcol) gsum[k] += unpack2<DT>((uint32_t)ra[i][k]);   // the rounded operand
            }
          }
        } else if constexpr (ABN) {   // dY = k1*dz + k2*y + k3 on the valid chunks (padding stays 0)
          if (av[i]) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const f32x2 dz = unpack2<DT>((uint32_t)ra[i][k]);
              const f32x2 yv = unpack2<DT>((uint32_t)ray[i][k]);
              ra[i][k] = (int)pack2<DT>(bnb_affine2(bk1[k], bk2[k], bk3[k], dz, yv));
            }
          }
        }
        const int ca = F32 ? col_addr_f32<BM>(tid / CPR + RPI * i, tid % CPR)
                           : col_addr<BM>(tid / CPR + RPI * i, tid % CPR);
        if constexpr (SPLIT) split_put(sa, ca, ra[i], ra2[i]);
        else *reinterpret_cast<i32x4*>(sa + ca) = ra[i];
      }
    }
    if constexpr (B_ROW) {
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        const int addr = row_addr((tid >> 3) + 32 * i, tid & 7);
        if constexpr (SPLIT) split_put(sb, addr, rb[i], rb2[i]);
        else *reinterpret_cast<i32x4*>(sb + addr) = rb[i];
      }
    } else {
      constexpr int CPR = BN / EPC, RPI = NT / CPR;
      if (gsame) return;
#pragma unroll
      for (int i = 0; i < BR; ++i) {
        if constexpr (PASS == WGRAD) {
          if constexpr (SPLIT) {
            if (pro && pv[i]) pro_apply2(rb[i], rb2[i]);
          } else {
            if (pro && pv[i]) pro_apply(rb[i]);
          }
        }
        const int cb_ = F32 ? col_addr_f32<BN>(tid / CPR + RPI * i, tid % CPR)
                            : col_addr<BN>(tid / CPR + RPI * i, tid % CPR);
        if constexpr (SPLIT) split_put(sb, cb_, rb[i], rb2[i]);
        else *reinterpret_cast<i32x4*>(sb + cb_) = rb[i];
      }
    }
  };

  // FWD_TAIL: write the staged activation chunks (and their ReLU bytes) of the k-tile in LDS,
  // read back from the tile image -- issued after the MFMAs, i.e. after the NEXT tile's loads: a
  // global store issued before those loads would hold their vmcnt wait behind its completion (VMEM
  // counts loads and stores in order), which made the in-staging store 4x slower per launch
  auto tail_store = [&]() __attribute__((always_inline)) {
    if constexpr (TAILP) {
      if (!tail_wr) return;
#pragma unroll
      for (int i = 0; i < AR; ++i) {
        if (!pv[i]) continue;   // 1x1 stride 1: row validity is the same for every k-tile
        const i32x4 v = *reinterpret_cast<const i32x4*>(smem + row_addr((tid >> 3) + 32 * i, tid & 7));
        const uint32_t e = (uint32_t)(a_base[i] / ES) + (uint32_t)(st_c_w + (tid & 7) * EPC);
        *reinterpret_cast<i32x4*>(reinterpret_cast<u16*>(p.pro_out) + e) = v;
        if (p.pro_mask) p.pro_mask[e >> 3] = (uint8_t)(tail_bits >> (8 * i));
      }
    }
  };

  // ---- LDS-DMA loader (DMA) ----------------------------------------------------------------
  // Piece j of a thread is the 16-B chunk q = (wid*G + j)*64 + lane of the operand tile's LDS
  // image, in LDS order (buffer_load ... lds writes lane-linearly at M0 + 16*lane). The images keep
  // the register path's XOR swizzles: they are applied to the SOURCE -- the slot of row/krow r holds
  // logical chunk slot ^ swz(r) -- so the fragment reads are the same code. Everything that does not
  // change along K is precomputed; a k-tile then costs 1-3 VALU per piece (FWD/DGRAD tap select,
  // an add) and, for the gathered WGRAD B, one pixel decode per piece.
  constexpr int GA = DMA ? A_BYTES / (NTH * 16) : 1, GB = DMA ? B_BYTES / (NTH * 16) : 1;
  static_assert(!DMA || (GA >= 1 && GB >= 1 && A_BYTES % (NTH * 16) == 0 &&
                         B_BYTES % (NTH * 16) == 0), "DMA tile");
  int da_base[GA];        // A ROW: byte offset of the row's tap-(0,0) pixel + chunk (may be < 0)
  uint64_t da_mask[GA];   // A ROW: taps of the row inside the image
  uint32_t da_off[GA];    // A COL (WGRAD): byte offset of (krow, col) at k = kbeg
  uint32_t db_off[GB];    // B at k = kbeg: FWD W row / DGRAD W k-row / WGRAD direct X row
  int db_c[GB], db_r[GB], db_s[GB], db_krow[GB];   // WGRAD gathered B: column (tap, c), k row
  bool db_ok[GB];
  constexpr int HA = HALO ? SLAB_ROWS / 64 : 1;     // HALO: slab pieces per thread and chunk
  uint32_t ha_off[HA];                               // HALO: slab piece sources at channel 0
  int hrow[HALO ? BM / WM / 16 : 1];                 // HALO: slab row of the fragment's pixel
  uint32_t hmask[HALO ? BM / WM / 16 : 1];           // HALO: taps inside the image (bit t)
  if constexpr (DMA) {
    const int rch = (lane & 7) ^ ((lane >> 3) & 7);   // ROW images: chunk of the lane's slot
    if constexpr (HALO) {
      // slab piece j: rows j*64 + wid*8 + lane/8 of the slab = pixels m0 - W - 1 + row
      const int csz = PASS == FWD ? p.Cin : p.Cout;
#pragma unroll
      for (int j = 0; j < HA; ++j) {
        const int pix = m0 - (p.W + 1) + j * 64 + wid * 8 + (lane >> 3);
        ha_off[j] = (pix >= 0 && pix < p.M) ? (uint32_t)(pix * csz + rch * 8) * (uint32_t)ES : OOB;
      }
      // fragment rows: slab row of the tap-centre pixel and the taps that stay inside the image
#pragma unroll
      for (int i = 0; i < BM / WM / 16; ++i) {
        const int rl = wr * (BM / WM) + i * 16 + (lane & 15);
        const int m = m0 + rl;
        hrow[i] = rl + p.W + 1;
        const uint32_t mm = m < p.M ? m : 0;
        const uint32_t img = fdiv(mm, p.dHoWo), rem = mm - img * p.dHoWo.d;
        const int y = (int)fdiv(rem, p.dWo), x = (int)(rem - (uint32_t)y * p.dWo.d);
        uint32_t msk = 0;
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int dy = PASS == FWD ? t / 3 - 1 : 1 - t / 3, dx = PASS == FWD ? t % 3 - 1 : 1 - t % 3;
          if ((unsigned)(y + dy) < (unsigned)p.H && (unsigned)(x + dx) < (unsigned)p.W) msk |= 1u << t;
        }
        hmask[i] = m < p.M ? msk : 0u;
      }
    } else if constexpr (A_ROW) {
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const int m = m0 + (wid * GA + j) * 8 + (lane >> 3);
        const bool okm = m < p.M;
        const uint32_t mm = okm ? m : 0;
        uint64_t msk = 0;
        int base;
        if constexpr (PASS == FWD) {
          const uint32_t img = fdiv(mm, p.dHoWo), rem = mm - img * p.dHoWo.d;
          const uint32_t yo = fdiv(rem, p.dWo), xo = rem - yo * p.dWo.d;
          const int y0 = (int)yo * p.stride - p.pad, x0 = (int)xo * p.stride - p.pad;
          base = (((int)img * p.H + y0) * p.W + x0) * p.Cin * ES;
          for (int r = 0, t = 0; r < p.R; ++r) {
            const bool yok = (unsigned)(y0 + r) < (unsigned)p.H;
            for (int q = 0; q < p.S; ++q, ++t)
              if (yok && (unsigned)(x0 + q) < (unsigned)p.W) msk |= 1ull << t;
          }
        } else {   // DGRAD class-grid pixel
          const uint32_t img = fdiv(mm, p.dHcWc), rem = mm - img * p.dHcWc.d;
          const uint32_t yi = fdiv(rem, p.dWc), xi = rem - yi * p.dWc.d;
          base = (((int)img * p.Ho + (int)yi) * p.Wo + (int)xi) * p.Cout * ES;
          for (int t = 0; t < ntap; ++t)
            if ((unsigned)((int)yi + p.tdy[split][t]) < (unsigned)p.Ho &&
                (unsigned)((int)xi + p.tdx[split][t]) < (unsigned)p.Wo)
              msk |= 1ull << t;
        }
        da_base[j] = base + rch * 16;
        da_mask[j] = okm ? msk : 0ull;
      }
    } else {   // WGRAD A: dY COL image [64 pixels][BM channels]
      constexpr int CPR = BM / 8;
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const int q = (wid * GA + j) * 64 + lane, krow = q / CPR;
        const int col = m0 + ((q % CPR) ^ col_swz<BM>(krow)) * 8;
        da_off[j] = col < p.M ? (uint32_t)((kbeg + krow) * p.Cout + col) * (uint32_t)ES : OOB;
      }
    }
    if constexpr (PASS == FWD) {   // B ROW: W [N][Kpad]
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int n = n0 + (wid * GB + j) * 8 + (lane >> 3);
        db_off[j] = n < p.N ? (uint32_t)(n * p.Kpad + rch * 8) * (uint32_t)ES : OOB;
      }
    } else {   // B COL [64 k][BN]
      constexpr int CPR = BN / 8;
#pragma unroll
      for (int j = 0; j < GB; ++j) {
        const int q = (wid * GB + j) * 64 + lane, krow = q / CPR;
        const int col = n0 + ((q % CPR) ^ col_swz<BN>(krow)) * 8;
        if constexpr (PASS == DGRAD) {   // W[cout = k][tap][cin = col]
          db_off[j] = col < p.N ? (uint32_t)(krow * p.R * p.S * p.Cin + col) * (uint32_t)ES : OOB;
        } else {                         // X gathered at column (tap, c)
          const int tap = col >> p.log2Cin;
          db_c[j] = col & ((1 << p.log2Cin) - 1);
          db_r[j] = (int)fdiv(tap, p.dS);
          db_s[j] = tap - db_r[j] * p.S;
          db_ok[j] = col < p.N && tap < p.R * p.S;
          db_krow[j] = krow;
          db_off[j] = db_ok[j] ? (uint32_t)((kbeg + krow) * p.Cin + db_c[j]) * (uint32_t)ES : OOB;
        }
      }
    }
  }
  // source offsets of the thread's pieces of k-tile kt: voff[0, GA) A, voff[GA, GA+GB) B
  constexpr int GP = GA + GB;
  auto dma_offsets = [&](int kt, uint32_t* voff) __attribute__((always_inline)) {
    const int k0 = kbeg + kt * BKE;
    if constexpr (PASS == FWD) {   // the k-tile lies in one tap (Cin a power of two >= 64)
      const int tap = k0 >> p.log2Cin;
      const int c0 = k0 & ((1 << p.log2Cin) - 1);
      const int r = (int)fdiv(tap, p.dS), q = tap - r * p.S;
      const int toff = ((r * p.W + q) * p.Cin + c0) * ES;
      const uint32_t word = tap >> 5, bit = tap & 31;
#pragma unroll
      for (int j = 0; j < GA; ++j) {
        const uint32_t mw = word ? (uint32_t)(da_mask[j] >> 32) : (uint32_t)da_mask[j];
        voff[j] = ((mw >> bit) & 1u) ? (uint32_t)(da_base[j] + toff) : OOB;
      }
#pragma unroll
      for (int j = 0; j < GB; ++j) voff[GA + j] = db_off[j] + (uint32_t)k0 * ES;
    } else if constexpr (PASS == DGRAD) {   // one tap per k-tile (Cout % 64 == 0)
      const int ti = p.log2Cout >= 0 ? k0 >> p.log2Cout : k0 / p.Cout;
      const int tsel = ti < 9 ? ti : 0;
      const int c = k0 - ti * p.Cout;
      const int toff = ((p.tdy[split][tsel] * p.Wo + p.tdx[split][tsel]) * p.Cout + c) * ES;
#pragma unroll
      for (int j = 0; j < GA; ++j)
        voff[j] = (((uint32_t)da_mask[j] >> ti) & 1u) ? (uint32_t)(da_base[j] + toff) : OOB;
      const uint32_t uoff = (uint32_t)((c * p.R * p.S + p.taps[split][tsel]) * p.Cin) * (uint32_t)ES;
#pragma unroll
      for (int j = 0; j < GB; ++j) voff[GA + j] = db_off[j] + uoff;
    } else {   // WGRAD: rows past the split's end (ragged last split) are past the buffers' end
      const uint32_t koff = (uint32_t)(kt * BKE * p.Cout) * (uint32_t)ES;
#pragma unroll
      for (int j = 0; j < GA; ++j) voff[j] = da_off[j] + koff;
      if (wb_direct) {
        const uint32_t xoff = (uint32_t)(kt * BKE * p.Cin) * (uint32_t)ES;
#pragma unroll
        for (int j = 0; j < GB; ++j) voff[GA + j] = db_off[j] + xoff;
      } else {
#pragma unroll
        for (int j = 0; j < GB; ++j) {
          const int m = k0 + db_krow[j];
          bool ok = db_ok[j] && m < kend;
          const uint32_t mm = ok ? m : 0;
          const uint32_t img = fdiv(mm, p.dHoWo), rem = mm - img * p.dHoWo.d;
          const uint32_t yo = fdiv(rem, p.dWo), xo = rem - yo * p.dWo.d;
          const int y = (int)yo * p.stride - p.pad + db_r[j], x = (int)xo * p.stride - p.pad + db_s[j];
          ok = ok && (unsigned)y < (unsigned)p.H && (unsigned)x < (unsigned)p.W;
          voff[GA + j] = ok ? (uint32_t)(((((int)img * p.H + y) * p.W + x) * p.Cin + db_c[j]) * ES) : OOB;
        }
      }
    }
  };
  // piece i of the thread into ring slot `slot`
  auto dma_piece = [&](int i, int slot, const uint32_t* voff) __attribute__((always_inline)) {
    char* sa = smem + slot * STAGE;
    if (i < GA) dma16(rsa, sa + (wid * GA + i) * 1024, voff[i]);
    else dma16(rsb, sa + A_BYTES + (wid * GB + i - GA) * 1024, voff[i]);
  };
  auto issue_dma = [&](int kt, int slot) __attribute__((always_inline)) {
    uint32_t voff[GP];
    dma_offsets(kt, voff);
#pragma unroll
    for (int i = 0; i < GP; ++i) dma_piece(i, slot, voff);
  };

  // acc[i][j][e] = C[wr*(BM/2) + i*16 + (lane&15)][wc*(BN/2) + j*16 + 4*(lane>>4) + e].
  // The MFMA runs with its operands swapped (per 16x16 tile D = Bfrag x Afrag^T = C^T), so every
  // lane ends up holding 4 consecutive COLUMNS of one row: the epilogue writes the C tile with one
  // 8-byte packed LDS store per MFMA tile (and the f32 paths with 16-byte stores) instead of
  // per-element 2-byte stores.
  constexpr int MI = BM / WM / 16, NI = BN / WN / 16;   // 16x16 tiles per wave
  f32x4 acc[MI][NI];
#pragma unroll
  for (int i = 0; i < MI; ++i)
#pragma unroll
    for (int j = 0; j < NI; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // MFMAs of one staged k-tile (A image at sa, B image at sb)
  auto mma_tile = [&](const char* sa, const char* sb) __attribute__((always_inline)) {
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      if constexpr (F32) {   // 16 k per step: lane holds 4 k of its row/col; 4 MFMAs 16x16x4 f32
        f32x4 fa[MI], fb[NI];
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int rbase = wr * (BM / WM) + i * 16;
          if constexpr (A_ROW) fa[i] = __builtin_bit_cast(f32x4, frag_row(sa, rbase, s, lane));
          else fa[i] = frag_col_f32<BM>(sa, rbase, s, lane);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cbase = wc * (BN / WN) + j * 16;
          if constexpr (B_ROW) fb[j] = __builtin_bit_cast(f32x4, frag_row(sb, cbase, s, lane));
          else fb[j] = frag_col_f32<BN>(sb, cbase, s, lane);
        }
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < MI; ++i)
#pragma unroll
            for (int j = 0; j < NI; ++j) acc[i][j] = mfma16_f32(fb[j][e], fa[i][e], acc[i][j]);
        continue;
      } else {
      s16x8 fa[MI], fb[NI];
#pragma unroll
      for (int i = 0; i < MI; ++i) {
        const int rbase = wr * (BM / WM) + i * 16;
        if constexpr (A_ROW) fa[i] = frag_row(sa, rbase, s, lane);
        else fa[i] = frag_col<BM>(sa, rbase, s, lane);
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const int cbase = wc * (BN / WN) + j * 16;
        if constexpr (B_ROW) fb[j] = frag_row(sb, cbase, s, lane);
        else fb[j] = frag_col<BN>(sb, cbase, s, lane);
      }
      if constexpr (SPLIT) {   // a*b ~ a_hi*b_hi + a_hi*b_lo + a_lo*b_hi
        s16x8 fl[NI > MI ? NI : MI];
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cbase = wc * (BN / WN) + j * 16;
          if constexpr (B_ROW) fl[j] = frag_row(sb + AB_BYTES, cbase, s, lane);
          else fl[j] = frag_col<BN>(sb + AB_BYTES, cbase, s, lane);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            acc[i][j] = mfma16<MDT>(fb[j], fa[i], acc[i][j]);
            acc[i][j] = mfma16<MDT>(fl[j], fa[i], acc[i][j]);
          }
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int rbase = wr * (BM / WM) + i * 16;
          if constexpr (A_ROW) fl[i] = frag_row(sa + AB_BYTES, rbase, s, lane);
          else fl[i] = frag_col<BM>(sa + AB_BYTES, rbase, s, lane);
        }
#pragma unroll
        for (int i = 0; i < MI; ++i)
#pragma unroll
          for (int j = 0; j < NI; ++j) acc[i][j] = mfma16<MDT>(fb[j], fl[i], acc[i][j]);
      } else {
      // data gradients (and the forward / folded-dgrad tiles up to 128x64): every fragment read
      // of the k-step issued before its MFMAs, so the compiler overlaps the next step's reads
      // with this step's MFMAs instead of re-using one A-fragment register (a read + wait per 4
      // MFMAs): -1..-6 % per data-gradient kernel in isolation, -0.08 ms/step more with the small
      // forward tiles (profiles/ab_r4.md sections 9-10; the 128x128 forward tiles would spill)
      if constexpr (!SPLIT && !F32 && (PASS_T == DGRAD || ((PASS_T == FWD || PASS_T == DGRAD_BNF) &&
                                                           BM * BN <= 128 * 64))) {
        __builtin_amdgcn_sched_group_barrier(0x100, MI + (B_ROW ? NI : 2 * NI) + (A_ROW ? 0 : MI), 0);
        __builtin_amdgcn_sched_group_barrier(0x008, MI * NI, 0);
      }
#pragma unroll
      for (int i = 0; i < MI; ++i)
#pragma unroll
        for (int j = 0; j < NI; ++j) acc[i][j] = mfma16<MDT>(fb[j], fa[i], acc[i][j]);
      }
      }
    }
  };

  if constexpr (HALO) {
    // Tap reuse (3x3, stride 1, pad 1): the k loop runs over (64-channel chunk cc, tap t). Per chunk
    // ONE slab of BM + 2W + 2 consecutive input rows (pixels m0-W-1 ..) is DMA'd into LDS; tap t
    // reads its A fragments from that slab shifted by the tap's pixel offset, and a row whose tap
    // falls outside the image reads the zero row instead. Only the weight tile streams per tap:
    // per 9 k-tiles the block takes in one slab + 9 weight tiles instead of 9 gathered A tiles.
    // Schedule: weight tile of step s+2 and one slab piece of chunk cc+1 (steps t < HA) are issued
    // during step s; a step starts with a counted vmcnt + ONE barrier (slot reuse as in the DMA
    // ring: weight slot (s+2)%3 = (s-1)%3, slab slot (cc+1)&1 last read in chunk cc-1).
    const int csz = PASS == FWD ? p.Cin : p.Cout;
    const int nch = csz >> 6;
    const int Wd = p.W;
    if (tid < 8) *reinterpret_cast<i32x4*>(smem + ZOFF + tid * 16) = i32x4{0, 0, 0, 0};
    auto a_piece = [&](int cc, int j) __attribute__((always_inline)) {
      dma16(rsa, smem + (cc & 1) * SLAB_BYTES + (j * 8 + wid) * 1024,
            cc < nch ? ha_off[j] + (uint32_t)(cc * 64 * ES) : OOB);
    };
    auto b_offsets = [&](int cc, int t, uint32_t* voff) __attribute__((always_inline)) {
      const uint32_t k = PASS == FWD ? (uint32_t)((t * p.Cin + cc * 64) * ES)
                                     : (uint32_t)((cc * 64 * p.R * p.S + t) * p.Cin * ES);
#pragma unroll
      for (int j = 0; j < GB; ++j) voff[j] = cc < nch ? db_off[j] + k : OOB;
    };
    auto b_piece = [&](int slot, int j, const uint32_t* voff) __attribute__((always_inline)) {
      dma16(rsb, smem + 2 * SLAB_BYTES + slot * B_BYTES + (wid * GB + j) * 1024, voff[j]);
    };
    {
#pragma unroll
      for (int j = 0; j < HA; ++j) a_piece(0, j);
      uint32_t v0[GB], v1[GB];
      b_offsets(0, 0, v0);
      b_offsets(0, 1, v1);
#pragma unroll
      for (int j = 0; j < GB; ++j) b_piece(0, j, v0);
#pragma unroll
      for (int j = 0; j < GB; ++j) b_piece(1, j, v1);
    }
    for (int cc = 0; cc < nch; ++cc) {
      const char* slab = smem + (cc & 1) * SLAB_BYTES;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        if (t >= 1 && t <= HA) vm_wait<GB + 1>(); else vm_wait<GB>();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_barrier();
        const int r = t / 3, q = t % 3;
        const int toff = PASS == FWD ? (r - 1) * Wd + (q - 1) : (1 - r) * Wd + (1 - q);
        const char* sb = smem + 2 * SLAB_BYTES + (t % 3) * B_BYTES;
        uint32_t voff[GB];
        b_offsets(t >= 7 ? cc + 1 : cc, t >= 7 ? t - 7 : t + 2, voff);
        constexpr int NMF = MI * NI;
        constexpr int NP = GB + 1;   // pieces of this step (the slab piece only while t < HA)
#pragma unroll
        for (int s2 = 0; s2 < 2; ++s2) {
          s16x8 fa[MI], fb[NI];
#pragma unroll
          for (int i = 0; i < MI; ++i) {
            const int row = hrow[i] + toff;
            const int chunk = s2 * 4 + (lane >> 4);
            const char* src = ((hmask[i] >> t) & 1u) ? slab + row * 128 + ((chunk ^ (row & 7)) << 4)
                                                     : smem + ZOFF;
            fa[i] = *reinterpret_cast<const s16x8*>(src);
          }
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const int cbase = wc * (BN / WN) + j * 16;
            if constexpr (B_ROW) fb[j] = frag_row(sb, cbase, s2, lane);
            else fb[j] = frag_col<BN>(sb, cbase, s2, lane);
          }
          // data gradients: the MFMA bursts at raised wave priority (-10..-12 % on the C10 / C16
          // tap-reuse dgrad in isolation; the forward lost 3-8 %: profiles/ab_r4.md section 11)
          if constexpr (PASS == DGRAD) __builtin_amdgcn_s_setprio(1);
#pragma unroll
          for (int idx = 0; idx < NMF; ++idx) {
            const int i = idx / NI, j = idx % NI;
            acc[i][j] = mfma16<MDT>(fb[j], fa[i], acc[i][j]);
            const int g = s2 * NMF + idx;
#pragma unroll
            for (int pc = 0; pc < NP; ++pc) {
              if (g != (pc * 2 * NMF) / NP) continue;
              if (pc < GB) b_piece((t + 2) % 3, pc, voff);
              else if (t < HA) a_piece(cc + 1, t);
            }
          }
          if constexpr (PASS == DGRAD) __builtin_amdgcn_s_setprio(0);
        }
      }
    }
  } else if constexpr (DMA) {
    // 3-slot ring: tile kt lives in slot kt % 3. Tile kt+2 is issued right after the barrier that
    // retires tile kt (each wave's counted vmcnt + the barrier: every wave's DMA of tile kt has
    // landed) and that proves every wave finished reading slot (kt+2) % 3 = (kt-1) % 3.
#pragma unroll
    for (int t = 0; t < NSLOT - 1; ++t)
      if (t < nk) issue_dma(t, t);
    int slot = 0;
    for (int kt = 0; kt < nk; ++kt) {
      // tile kt must have landed: the younger tiles kt+1 .. kt+NSLOT-2 may stay in flight
      if constexpr (NSLOT == 4) {
        if (kt + 2 < nk) vm_wait<2 * GP>(); else if (kt + 1 < nk) vm_wait<GP>(); else vm_wait<0>();
      } else if constexpr (NSLOT == 3) {
        if (kt + 1 < nk) vm_wait<GP>(); else vm_wait<0>();
      } else {   // two slots: only tile kt is in flight here
        vm_wait<0>();
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      const int nslot = slot == 0 ? NSLOT - 1 : slot - 1;   // = (kt + NSLOT - 1) % NSLOT
      const char* sa = smem + slot * STAGE;
      const char* sb = sa + A_BYTES;
      // the pieces of tile kt+2 spread over this tile's MFMAs (a burst of LDS-DMA issues right
      // after the barrier holds every wave's matrix pipe: +10-20 % time, profiles/ab_r3_dma.md);
      // past the last tile they are OOB no-ops (nothing reads that slot again), so the MFMA
      // stream carries no branch
      uint32_t voff[GP];
      dma_offsets(kt + NSLOT - 1, voff);
      const bool pre = kt + NSLOT - 1 < nk;
#pragma unroll
      for (int i = 0; i < GP; ++i) voff[i] = pre ? voff[i] : OOB;
      constexpr int NMF = MI * NI;
      constexpr int NKS = BKE / 32;   // MFMA k-steps per tile
      // the fragments of k-step s+1 are read while the MFMAs of step s run (register double
      // buffer), and the MFMA bursts of 64-deep tiles run at raised wave priority: -3..-11 % on the
      // 128x256 / 256x128 weight-gradient tiles in isolation (profiles/ab_r4.md section 9)
      s16x8 fa[2][MI], fb[2][NI];
      auto ldf = [&](int s, int b) __attribute__((always_inline)) {
#pragma unroll
        for (int i = 0; i < MI; ++i) {
          const int rbase = wr * (BM / WM) + i * 16;
          if constexpr (A_ROW) fa[b][i] = frag_row(sa, rbase, s, lane);
          else fa[b][i] = frag_col<BM>(sa, rbase, s, lane);
        }
#pragma unroll
        for (int j = 0; j < NI; ++j) {
          const int cbase = wc * (BN / WN) + j * 16;
          if constexpr (B_ROW) fb[b][j] = frag_row(sb, cbase, s, lane);
          else fb[b][j] = frag_col<BN>(sb, cbase, s, lane);
        }
      };
      ldf(0, 0);
#pragma unroll
      for (int s = 0; s < NKS; ++s) {
        if (s + 1 < NKS) ldf(s + 1, (s + 1) & 1);
        if constexpr (NKS > 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int idx = 0; idx < NMF; ++idx) {
          const int i = idx / NI, j = idx % NI;
          acc[i][j] = mfma16<MDT>(fb[s & 1][j], fa[s & 1][i], acc[i][j]);
          const int g = s * NMF + idx;   // piece pc goes after MFMA (pc * NKS * NMF) / GP
#pragma unroll
          for (int pc = 0; pc < GP; ++pc)
            if (g == (pc * NKS * NMF) / GP) dma_piece(pc, nslot, voff);
        }
        if constexpr (NKS > 1) __builtin_amdgcn_s_setprio(0);
      }
      slot = slot == NSLOT - 1 ? 0 : slot + 1;
    }
  }
  if constexpr (DMA) {
    vm_wait<0>();
    __syncthreads();   // the epilogue reuses the ring
  } else {
    if (nk > 0) {
      load_tile(0);
      if constexpr (STAGES == 2) {
        store_tile(0);
        __syncthreads();
      }
    }
    for (int kt = 0; kt < nk; ++kt) {
      const int cur = STAGES == 2 ? (kt & 1) : 0;
      if constexpr (STAGES == 1) {   // registers hold tile kt: publish it, then prefetch kt+1
        store_tile(0);
        __syncthreads();
      }
      if (kt + 1 < nk) load_tile(kt + 1);
      const char* sa = smem + cur * STAGE;
      mma_tile(sa, gsame ? sa : sa + A_BYTES);
      if constexpr (STAGES == 2) {
        if (kt + 1 < nk) store_tile(cur ^ 1);
      }
      tail_store();
      __syncthreads();
    }
  }

  // ================================================================ epilogue
  const int lr = lane & 15, lg = lane >> 4;
  // every accumulator value as (row, 4 consecutive columns) within the wave tile: the MFMA runs
  // with swapped operands (D = C^T), so a lane holds 4 consecutive C columns per 16x16 tile
  auto for_items = [&](auto&& fn) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < NI; ++j)   // column-tile outer: measured ~1% faster FWD than row-outer
#pragma unroll
      for (int i = 0; i < MI; ++i) fn(i * 16 + lr, j * 16 + 4 * lg, acc[i][j]);
  };

  if constexpr (PASS == WGRAD) {
    // (WGRAD_GRAM: per split an [M + 1][N] block -- the partial Gram, then the column sums)
    float* slab = reinterpret_cast<float*>(p.out) + (size_t)split * (GRAM ? p.M + 1 : p.M) * p.N;
    const bool vec = (p.N & 3) == 0;
    for_items([&](int rl, int cl, const f32x4& v) {
      const int row = m0 + wr * (BM / WM) + rl;
      const int col = n0 + wc * (BN / WN) + cl;
      if (row >= p.M) return;
      float* d = slab + (size_t)row * p.N + col;
      if (vec) {
        if (col < p.N) *reinterpret_cast<f32x4*>(d) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (col + e < p.N) d[e] = v[e];
      }
    });
    if constexpr (GRAM) {   // column-sum partials of this split: row M of its block
      if (gcol) {
        constexpr int CPR = BM / EPC, RPI = NT / CPR;
        float* red = reinterpret_cast<float*>(smem);   // [RPI][BM] (the main loop is done with LDS)
        __syncthreads();
#pragma unroll
        for (int k = 0; k < 4; ++k)
          *reinterpret_cast<f32x2*>(red + (tid / CPR) * BM + (tid % CPR) * EPC + 2 * k) = gsum[k];
        __syncthreads();
        if (tid < BM && m0 + tid < p.M) {
          float a = 0.f;
          for (int g = 0; g < RPI; ++g) a += red[g * BM + tid];
          slab[(size_t)p.M * p.N + m0 + tid] = a;
        }
      }
    }
    return;
  } else {
    if (p.out_f32) {  // fc logits: f32 + bias, direct stores
      float* out = reinterpret_cast<float*>(p.out);
      for_items([&](int rl, int cl, const f32x4& v) {
        const int row = m0 + wr * (BM / WM) + rl;
        const int col = n0 + wc * (BN / WN) + cl;
        if (row >= p.M) return;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int c = col + e;
          if (c < p.N) out[(size_t)row * p.out_pitch + c] = v[e] + (p.bias ? p.bias[c] : 0.f);
        }
      });
      return;
    }
    const bool relu = p.relu != 0;
    // stage the C tile through LDS: [BM][BN], row pitch BN*ES bytes, 16-B chunks swizzled by
    // row; one packed 8-byte store (4 columns) per item per lane (f32: one 16-B store).
    constexpr int CPR = BN / EPO;
    auto c_addr = [&](int row, int chunk) { return row * CPR + (chunk ^ (row & (CPR - 1))); };
    // 16-bit C tile with BN <= 128: 8-byte pieces (4 columns) XOR-swizzled by cswz(row) instead of
    // 16-byte chunks. The MFMA layout writes one piece per lane and a ds_write_b64 lane group is 16
    // rows of ONE piece: 16-B chunks give them only 8 distinct bank quads (2-way conflicts on every
    // C-tile write -- the bulk of the 21-35 % LDS conflicts of the layer-1/2 launches,
    // profiles/pmc_r5_step.md); pieces give 16, i.e. all 32 banks. The reader loads its chunk as two
    // ds_read_b64 (same LDS cycles as one b128): conflict-free when rows 2 apart (BN = 64, 128-B
    // rows) or 1 apart (BN = 128) differ in the swizzle's parity.
    constexpr bool PIECE = !O32 && BN <= 128;
    auto cswz = [&](int row) __attribute__((always_inline)) {
      if constexpr (BN == 64) return (row & 12) | ((row & 1) << 1) | ((row >> 1) & 1);
      else return row & 15;
    };
    auto ld_c = [&](int row, int chunk) __attribute__((always_inline)) -> i32x4 {
      if constexpr (PIECE) {
        const char* rb = smem + row * (BN * ES);
        const int o = ((2 * chunk) ^ cswz(row)) << 3;
        const uint2 a = *reinterpret_cast<const uint2*>(rb + o);
        const uint2 b = *reinterpret_cast<const uint2*>(rb + (o ^ 8));
        return i32x4{(int)a.x, (int)a.y, (int)b.x, (int)b.y};
      } else {
        return *reinterpret_cast<const i32x4*>(smem + c_addr(row, chunk) * 16);
      }
    };
    // f32: the waves of wave-row h write their tiles to local rows [0, BM/2) of the LDS image
    auto stage_f32 = [&](int h) __attribute__((always_inline)) {
      if (wr != h) return;
      for_items([&](int rl, int cl, f32x4 v) {
        const int col = wc * (BN / WN) + cl;
        if (relu) v = __builtin_elementwise_max(v, (f32x4){0.f, 0.f, 0.f, 0.f});
        *reinterpret_cast<f32x4*>(smem + rl * (BN * 4) + (((col >> 2) ^ (rl & (CPR - 1))) << 4)) = v;
      });
    };
    if constexpr (!O32) {
      for_items([&](int rl, int cl, f32x4 v) {
        const int col = wc * (BN / WN) + cl;
        const int row = wr * (BM / WM) + rl;
        if constexpr (BNF) {   // b = W^T k3 where the class has a tap (a 1x1 conv's landing pixels)
          if (ntap > 0 && n0 + col < p.N) v += *reinterpret_cast<const f32x4*>(p.dbias + n0 + col);
        }
        if (relu) v = __builtin_elementwise_max(v, (f32x4){0.f, 0.f, 0.f, 0.f});
        // row & (CPR-1) == lr & (CPR-1) for CPR <= 16 (folded); BN = 256 needs the full row
        const int cbyte = PIECE ? (((col >> 2) ^ cswz(row)) << 3)
                                : (((col >> 3) ^ (row & (CPR - 1))) << 4) + ((col & 4) << 1);
        uint2 pk;
        pk.x = pack2<DT>(f32x2{v[0], v[1]});
        pk.y = pack2<DT>(f32x2{v[2], v[3]});
        *reinterpret_cast<uint2*>(smem + row * (BN * 2) + cbyte) = pk;
      });
    }
    const char* ct = smem;
    // coalesced 16-B stores + per-channel partial statistics.
    //  FWD  (stats): q0 = sum y, q1 = sum y^2 of the written tile (BatchNorm forward statistics).
    //  DGRAD (emode >= 0): the tile is dA, the gradient of a = relu(bn(y) [+ res | + bn2(y2)]);
    //        the epilogue adds g2 (second gradient source), applies the ReLU mask recomputed from
    //        y (and the residual), stores dz instead of dA and emits q0 = sum dz, q1 = sum dz*y,
    //        q2 = sum dz*y2 -- the BatchNorm-backward reduction, with no extra pass over dA.
    // The BN mode and the g2 source are compile-time in the row loop (one uniform dispatch below),
    // and all per-element math runs on packed pairs (v_pk_fma_f32 / v_cvt_pk_*); unlike the operand
    // prologue, the packed form measured faster here.
    const int cc = tid % CPR;          // column chunk
    const int rg = tid / CPR;          // row group
    constexpr int RG = NTH / CPR;      // row groups
    constexpr int RPT = BM / RG;       // rows per thread
    constexpr int RPTH = RPT / NH;     // ... per staged half
    // rows are processed in groups of PD; the fused-epilogue operands of a group are loaded
    // before it is consumed (the first group's before the barrier that publishes the C tile),
    // which bounds the prefetch registers to PD rows.
    constexpr int PD = RPTH > 4 ? 4 : RPTH;
    char* outb = reinterpret_cast<char*>(p.out);
    const int gcol = n0 + cc * EPO;
    auto row_off = [&](int i, bool& ok) __attribute__((always_inline)) -> uint32_t {
      const int grow = m0 + rg + RG * i;
      ok = grow < p.M && gcol < p.N;
      uint32_t orow = ok ? grow : 0;
      if constexpr (PASS == DGRAD) {
        const uint32_t img = fdiv(orow, p.dHcWc), rem = orow - img * p.dHcWc.d;
        const uint32_t yi = fdiv(rem, p.dWc), xi = rem - yi * p.dWc.d;
        const int h = (int)yi * p.stride + cls_ph, w = (int)xi * p.stride + cls_pw;
        orow = ((uint32_t)img * p.H + h) * p.W + w;
      }
      return orow * (uint32_t)p.out_pitch + gcol;
    };

    auto rows = [&](auto mode_c, auto g2_c) __attribute__((always_inline)) {
      constexpr int MODE = decltype(mode_c)::value;   // -1 plain / FWD stats; 0,1,2 BN-backward
      constexpr bool G2 = decltype(g2_c)::value != 0;
      constexpr int NQ = MODE == 2 ? 3 : 2;
      const bool do_stats = MODE >= 0 || (PASS == FWD && p.stats != nullptr);
      constexpr bool Y2 = MODE == 1 || MODE == 2;   // residual / shortcut tensor read
      f32x2 esc[4], esh[4], esc2[4], esh2[4];
      if constexpr (MODE >= 0 && MODE != 3) {
        const int cg = gcol < p.N ? gcol : 0;
#pragma unroll
        for (int k = 0; k < EPO / 2; ++k) {
          esc[k] = f32x2{p.esc[cg + 2 * k], p.esc[cg + 2 * k + 1]};
          esh[k] = f32x2{p.esh[cg + 2 * k], p.esh[cg + 2 * k + 1]};
          if constexpr (MODE == 2) {
            esc2[k] = f32x2{p.esc2[cg + 2 * k], p.esc2[cg + 2 * k + 1]};
            esh2[k] = f32x2{p.esh2[cg + 2 * k], p.esh2[cg + 2 * k + 1]};
          }
        }
      }
      uint32_t eoff[PD];
      bool eok[PD];
      i32x4 py[PD], pg2[PD], py2[PD];
      uint32_t pm[PD];
      auto prefetch = [&](int g0) __attribute__((always_inline)) {
        const i32x4 z = {0, 0, 0, 0};
#pragma unroll
        for (int j = 0; j < PD; ++j) {
          eoff[j] = row_off(g0 + j, eok[j]);
          const size_t bo = (size_t)eoff[j] * ES;
          auto ld = [&](const void* base) __attribute__((always_inline)) {
            const i32x4* q = reinterpret_cast<const i32x4*>(reinterpret_cast<const char*>(base) + bo);
            return *q;
          };
          if constexpr (MODE >= 0) py[j] = eok[j] ? ld(p.ey) : z;
          if constexpr (G2) pg2[j] = eok[j] ? ld(p.eg2) : z;
          if constexpr (Y2) py2[j] = eok[j] ? ld(p.ey2) : z;
          if constexpr (MODE == 3) pm[j] = eok[j] ? (uint32_t)p.emask[eoff[j] >> 3] >> (eoff[j] & 7) : 0u;
        }
      };
      f32x2 q0[4], q1[4], q2[4], shv[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        q0[k] = f32x2{0.f, 0.f}; q1[k] = q0[k]; q2[k] = q0[k]; shv[k] = q0[k];
      }
      constexpr bool SHIFTED = PASS == FWD && MODE < 0;   // forward statistics: shifted sums
#pragma unroll
      for (int h = 0; h < NH; ++h) {
      if constexpr (O32) {
        if (h > 0) __syncthreads();   // every thread is done reading the previous half
        stage_f32(h);
      }
      prefetch(h * RPTH);
      __syncthreads();
      if (SHIFTED && h == 0 && do_stats) {   // shift = the tile's first row (always a valid row)
        const i32x4 v0 = ld_c(0, cc);
        if constexpr (O32) {
#pragma unroll
          for (int e = 0; e < 4; ++e) shv[e >> 1][e & 1] = __int_as_float(v0[e]);
        } else {
#pragma unroll
          for (int k = 0; k < 4; ++k) shv[k] = unpack2<DT>((uint32_t)v0[k]);
        }
      }
#pragma unroll
      for (int g0 = 0; g0 < RPTH; g0 += PD) {
        if (g0 > 0) prefetch(h * RPTH + g0);
#pragma unroll
        for (int j = 0; j < PD; ++j) {
          const int row = rg + RG * (g0 + j);   // local row of the staged half
          i32x4 v = ld_c(row, cc);
          if (!eok[j]) continue;
          if constexpr (O32) {   // one element per dword
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const int k = e >> 1, h = e & 1;
              float f = __int_as_float(v[e]);
              if constexpr (MODE >= 0) {
                if constexpr (G2) f += __int_as_float(pg2[j][e]);
                const float yv = __int_as_float(py[j][e]);
                float y2v = 0.f, dz;
                if constexpr (MODE == 3) {
                  dz = ((pm[j] >> e) & 1u) ? f : 0.f;
                } else {
                  float pre = yv * esc[k][h] + esh[k][h];
                  if constexpr (Y2) y2v = __int_as_float(py2[j][e]);
                  if constexpr (MODE == 1) pre += y2v;
                  if constexpr (MODE == 2) pre += y2v * esc2[k][h] + esh2[k][h];
                  dz = pre > 0.f ? f : 0.f;
                }
                v[e] = __float_as_int(dz);
                q0[k][h] += dz;
                q1[k][h] += dz * yv;
                if constexpr (MODE == 2) q2[k][h] += dz * y2v;
              } else if (do_stats) {
                const float dlt = f - shv[k][h];
                q0[k][h] += dlt;
                q1[k][h] += dlt * dlt;
              }
            }
          } else if constexpr (MODE >= 0) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              f32x2 g = unpack2<DT>((uint32_t)v[k]);
              if constexpr (G2) g += unpack2<DT>((uint32_t)pg2[j][k]);
              const f32x2 yv = unpack2<DT>((uint32_t)py[j][k]);
              f32x2 y2v = f32x2{0.f, 0.f}, dz;
              if constexpr (MODE == 3) {
                const uint32_t mb = pm[j] >> (2 * k);
                dz = f32x2{(mb & 1u) ? g.x : 0.f, (mb & 2u) ? g.y : 0.f};
              } else {
                f32x2 pre = yv * esc[k] + esh[k];
                if constexpr (Y2) y2v = unpack2<DT>((uint32_t)py2[j][k]);
                if constexpr (MODE == 1) pre += y2v;
                if constexpr (MODE == 2) pre += y2v * esc2[k] + esh2[k];
                dz = f32x2{pre.x > 0.f ? g.x : 0.f, pre.y > 0.f ? g.y : 0.f};
              }
              const uint32_t o = pack2<DT>(dz);
              if constexpr (G2) dz = unpack2<DT>(o);   // statistics of the stored (rounded) dz
              v[k] = (int)o;
              q0[k] += dz;
              q1[k] += dz * yv;
              if constexpr (MODE == 2) q2[k] += dz * y2v;
            }
          } else if (do_stats) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
              const f32x2 dlt = unpack2<DT>((uint32_t)v[k]) - shv[k];
              q0[k] += dlt;
              q1[k] += dlt * dlt;
            }
          }
          i32x4* dst = reinterpret_cast<i32x4*>(outb + (size_t)eoff[j] * ES);
          *dst = v;
        }
      }
      }
      if (do_stats) {
        __syncthreads();
        float* red = reinterpret_cast<float*>(smem);  // [NQ][RG][BN] (+ FWD: shift row)
        // column pair k of chunk cc sits at slot (k + cc/4 + 2*(row&1)) & 3 of the chunk's 8 floats:
        // the 16 lanes of one ds_write_b64 group (16 chunks of a row, or 8 chunks of two rows when
        // BN = 64) then cover all 32 banks -- the plain layout put 4 lanes on every bank pair
        auto spos = [&](int cc_, int k_, int g_) __attribute__((always_inline)) {
          if constexpr (EPO == 8) return cc_ * 8 + 2 * ((k_ + (cc_ >> 2) + 2 * (g_ & 1)) & 3);
          else return cc_ * EPO + 2 * k_;
        };
#pragma unroll
        for (int k = 0; k < EPO / 2; ++k) {
          const int sp = spos(cc, k, rg);
          *reinterpret_cast<f32x2*>(red + rg * BN + sp) = q0[k];
          *reinterpret_cast<f32x2*>(red + RG * BN + rg * BN + sp) = q1[k];
          if constexpr (NQ > 2) *reinterpret_cast<f32x2*>(red + 2 * RG * BN + rg * BN + sp) = q2[k];
          if constexpr (SHIFTED) {
            if (rg == 0) *reinterpret_cast<f32x2*>(red + 2 * RG * BN + spos(cc, k, 0)) = shv[k];
          }
        }
        __syncthreads();
        if (tid < BN) {
          float a = 0.f, b = 0.f, c2 = 0.f;
          // this thread's column in the even / odd rows of the swizzled layout
          const int e_ = tid % EPO;
          const int pe = spos(tid / EPO, e_ >> 1, 0) + (e_ & 1);
          const int po = spos(tid / EPO, e_ >> 1, 1) + (e_ & 1);
#pragma unroll 8
          for (int g = 0; g < RG; ++g) {
            const int pc = (g & 1) ? po : pe;
            a += red[g * BN + pc];
            b += red[RG * BN + g * BN + pc];
            if constexpr (NQ > 2) c2 += red[2 * RG * BN + g * BN + pc];
          }
          const int col = n0 + tid;
          if (col < p.N) {
            if constexpr (SHIFTED) {   // (sum d, sum d^2, shift)
              float* dst = p.stats + (size_t)tm * 3 * p.N + col;
              dst[0] = a;
              dst[p.N] = b;
              dst[2 * p.N] = red[2 * RG * BN + pe];
            } else {
              float* dst = p.epart;
              const size_t slab = (size_t)split * tiles_m + tm;
              dst[(slab * NQ + 0) * p.N + col] = a;
              dst[(slab * NQ + 1) * p.N + col] = b;
              if constexpr (NQ > 2) dst[(slab * NQ + 2) * p.N + col] = c2;
            }
          }
        }
      }
    };
    if constexpr (PASS == DGRAD) {
      const bool g2 = p.eg2 != nullptr;
      if (p.emode < 0) rows(IC<-1>{}, IC<0>{});
      else if (p.emode == 0) { if (g2) rows(IC<0>{}, IC<1>{}); else rows(IC<0>{}, IC<0>{}); }
      else if (p.emode == 1) { if (g2) rows(IC<1>{}, IC<1>{}); else rows(IC<1>{}, IC<0>{}); }
      else if (p.emode == 3) { if (g2) rows(IC<3>{}, IC<1>{}); else rows(IC<3>{}, IC<0>{}); }
      else { if (g2) rows(IC<2>{}, IC<1>{}); else rows(IC<2>{}, IC<0>{}); }
    } else {
      rows(IC<-1>{}, IC<0>{});
    }
  }
}

// split-K slab reduction for WGRAD, with layout remap + scale, into the f32 gradient buffer:
// grad[n1 * dst_pitch + (n2 / cin_pad) * cin_real + n2 % cin_pad] = scale * sum_s slab[s][n1][n2]
// for n2 % cin_pad < cin_real (stem: Cin padded 3 -> 8).
// Optional combine (ck != null, the decomposed tail-fold weight gradient): the summed value s of
// (row n1, column n2) becomes ck[n1] * s + ck[M + n1] * cB[n1 * N + n2] + ck[2M + n1] * cs[n2].
__device__ __forceinline__ float wg_combine(float s, const float* ck, const float* cB, const float* cs,
                                            int M, int N, int n1, int n2) {
  if (!ck) return s;
  return ck[n1] * s + ck[M + n1] * cB[(size_t)n1 * N + n2] + ck[2 * M + n1] * cs[n2];
}

__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, float* __restrict__ grad,
                                    int splits, int M, int N, int cin_pad_log2, int cin_real,
                                    int dst_pitch, float scale, int accumulate,
                                    const float* __restrict__ ck, const float* __restrict__ cB,
                                    const float* __restrict__ cs) {
  const int total = M * N;
  for (int idx = blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < splits; ++k) s += slab[(size_t)k * total + idx];
    const int n1 = idx / N, n2 = idx - n1 * N;
    s = wg_combine(s, ck, cB, cs, M, N, n1, n2);
    const int tap = n2 >> cin_pad_log2, c = n2 & ((1 << cin_pad_log2) - 1);
    if (c < cin_real) {
      float* d = grad + (size_t)n1 * dst_pitch + tap * cin_real + c;
      *d = accumulate ? *d + scale * s : scale * s;
    }
  }
}

// Parallel split-K reduction (N % 4 == 0): a block owns EPB consecutive elements and all splits;
// its 256 threads are SG = 256/(EPB/4) split groups x EPB/4 float4 columns, each group summing
// splits sg, sg+SG, ... then a fixed-order LDS combine -> deterministic. Small weight tiles with
// hundreds of splits (e.g. 64x64 1x1 convs) no longer serialise on one thread per element.
template <int EPB>
__global__ __launch_bounds__(256) void wgrad_reduce4_kernel(const float* __restrict__ slab,
                                                            float* __restrict__ grad, int splits,
                                                            int M, int N, int cin_pad_log2,
                                                            int cin_real, int dst_pitch, float scale,
                                                            int accumulate, const float* __restrict__ ck,
                                                            const float* __restrict__ cB,
                                                            const float* __restrict__ cs) {
  constexpr int TPE = EPB / 4, SG = 256 / TPE;
  __shared__ f32x4 red[256];
  const int total = M * N;
  const int t = threadIdx.x, sg = t / TPE, e4 = t - sg * TPE;
  const int base = blockIdx.x * EPB + e4 * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (base < total) {
    const float* src = slab + base;
#pragma unroll 4
    for (int k = sg; k < splits; k += SG) acc += *reinterpret_cast<const f32x4*>(src + (size_t)k * total);
  }
  red[t] = acc;
  __syncthreads();
  if (sg != 0 || base >= total) return;
  f32x4 s = red[e4];
  for (int g = 1; g < SG; ++g) s += red[g * TPE + e4];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = base + q;
    const int n1 = idx / N, n2 = idx - n1 * N;
    const int tap = n2 >> cin_pad_log2, c = n2 & ((1 << cin_pad_log2) - 1);
    if (c < cin_real) {
      const float v = wg_combine(s[q], ck, cB, cs, M, N, n1, n2);
      float* d = grad + (size_t)n1 * dst_pitch + tap * cin_real + c;
      *d = accumulate ? *d + scale * v : scale * v;
    }
  }
}


// Several split-K reductions in ONE launch (the weight gradients of a whole stage, queued by
// native_ops.ReduceBatch): block b serves descriptor k with blk0[k] <= b < blk0[k+1], then runs
// wgrad_reduce4_kernel<64>'s fixed-order sum (16 split groups x 16 float4 columns, LDS combine in
// group order: deterministic) with that descriptor's remap / scale / combine.
constexpr int RB_MAX = 24;
struct RedDesc {
  const float* slab; float* grad; const float* ck; const float* cB; const float* cs;
  int splits, M, N, cin_log2, cin_real, pitch, accumulate, blk0;
  float scale;
};
struct RedBatch {
  int n;
  RedDesc d[RB_MAX];
};
__global__ __launch_bounds__(256) void wgrad_reduce_batch_kernel(RedBatch b_arg) {
#if defined(__HIP_DEVICE_COMPILE__)
  typedef const __attribute__((address_space(4))) RedBatch KB;
  KB& b = *(KB*)__builtin_amdgcn_kernarg_segment_ptr();
#else
  const RedBatch& b = b_arg;
#endif
  const int bid = blockIdx.x;
  int k = 0;
  while (k + 1 < b.n && bid >= b.d[k + 1].blk0) ++k;
  const float* slab = b.d[k].slab;
  const int M = b.d[k].M, N = b.d[k].N, splits = b.d[k].splits;
  constexpr int EPB = 64, TPE = EPB / 4, SG = 256 / TPE;
  __shared__ f32x4 red[256];
  const int total = M * N;
  const int t = threadIdx.x, sg = t / TPE, e4 = t - sg * TPE;
  const int base = (bid - b.d[k].blk0) * EPB + e4 * 4;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  if (base < total) {
    const float* src = slab + base;
#pragma unroll 4
    for (int s = sg; s < splits; s += SG) acc += *reinterpret_cast<const f32x4*>(src + (size_t)s * total);
  }
  red[t] = acc;
  __syncthreads();
  if (sg != 0 || base >= total) return;
  f32x4 sum = red[e4];
  for (int g = 1; g < SG; ++g) sum += red[g * TPE + e4];
  const int cl = b.d[k].cin_log2, cr = b.d[k].cin_real, pitch = b.d[k].pitch;
  const float scale = b.d[k].scale;
  const bool accumulate = b.d[k].accumulate != 0;
  float* grad = b.d[k].grad;
  const float *ck = b.d[k].ck, *cB = b.d[k].cB, *cs = b.d[k].cs;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int idx = base + q;
    const int n1 = idx / N, n2 = idx - n1 * N;
    const int tap = n2 >> cl, c = n2 & ((1 << cl) - 1);
    if (c < cr) {
      const float v = wg_combine(sum[q], ck, cB, cs, M, N, n1, n2);
      float* d = grad + (size_t)n1 * pitch + tap * cr + c;
      *d = accumulate ? *d + scale * v : scale * v;
    }
  }
}

// Consumer-side BatchNorm-backward fold (DGRAD_BNF operands) in ONE launch. W: the conv's 16-bit
// weights [Cout][Cin] (1x1, OHWI); k: [k1; k2; k3] (3 x Cout f32, the BN-backward apply
// coefficients of the BN after the conv). Writes Wf = [k1 o W ; G] ([Cout + Cin][Cin] 16-bit),
// G = W^T diag(k2) W, and b = W^T k3 (f32 [Cin]).
// Three block roles in one grid:
//   G    : one 16x16 tile of G per block; its 4 waves take every 4th 32-deep k-step of K = Cout and
//          load their MFMA 16x16x32 fragments straight from W (lane: column l&15 of the panel, rows
//          8(l>>4)..+7 of the k-step -- W is a few hundred KiB, L2-resident), the B operand scaled
//          by k2 and rounded to 16 bits once; the 4 partials are summed in wave order through LDS;
//   bias : one wave per column i, lanes strided over K, a fixed xor-butterfly combine;
//   rows : k1 o W, one 16-B chunk per thread.
// No LDS tile images (4 KiB of LDS): the launch runs on the main stream beside the weight-gradient
// LDS-DMA tiles (144 KiB of a CU's 160 KiB). The tiled 96 KiB form took 11-17 us per launch with a
// 188 us outlier when it had to wait for a CU without one. Deterministic.
template <int DT>
__global__ __launch_bounds__(256) void bn_fold_kernel(const u16* __restrict__ W,
                                                      const float* __restrict__ k, int Cout, int Cin,
                                                      u16* __restrict__ Wf, float* __restrict__ bias,
                                                      int nG, int nB) {
  __shared__ __attribute__((aligned(16))) f32x4 red[4][64];
  const float* k1 = k;
  const float* k2 = k + Cout;
  const float* k3 = k + 2 * Cout;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  int b = blockIdx.x;
  if (b < nG) {   // ---- G tile (ti, tj)
    const int n16 = Cin >> 4;
    const int ti = b / n16, tj = b - ti * n16;
    const int r = lane & 15, g = lane >> 4;
    const u16* pa = W + ti * 16 + r;
    const u16* pb = W + tj * 16 + r;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    const int nks = Cout >> 5;
#pragma unroll 2
    for (int s = wid; s < nks; s += 4) {
      const int k0 = s * 32 + 8 * g;
      const f32x4 q0 = *reinterpret_cast<const f32x4*>(k2 + k0);
      const f32x4 q1 = *reinterpret_cast<const f32x4*>(k2 + k0 + 4);
      uint32_t ua[8], ub[8];
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        ua[e] = pa[(size_t)(k0 + e) * Cin];
        ub[e] = pb[(size_t)(k0 + e) * Cin];
      }
      s16x8 fa, fb;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const uint32_t pa2 = ua[2 * q] | (ua[2 * q + 1] << 16);
        const f32x2 f = unpack2<DT>(ub[2 * q] | (ub[2 * q + 1] << 16));
        const float s0 = q < 2 ? q0[2 * q] : q1[2 * q - 4];
        const float s1 = q < 2 ? q0[2 * q + 1] : q1[2 * q - 3];
        const uint32_t pb2 = pack2<DT>(f32x2{f.x * s0, f.y * s1});
        fa[2 * q] = (short)(pa2 & 0xffff); fa[2 * q + 1] = (short)(pa2 >> 16);
        fb[2 * q] = (short)(pb2 & 0xffff); fb[2 * q + 1] = (short)(pb2 >> 16);
      }
      acc = mfma16<DT>(fb, fa, acc);
    }
    // acc[e] = partial G[ti*16 + r][tj*16 + 4g + e]; waves 1-3 hand theirs to wave 0
    red[wid][lane] = acc;
    __syncthreads();
    if (wid == 0) {
      const f32x4 v = ((red[0][lane] + red[1][lane]) + red[2][lane]) + red[3][lane];
      uint2 pk;
      pk.x = pack2<DT>(f32x2{v[0], v[1]});
      pk.y = pack2<DT>(f32x2{v[2], v[3]});
      *reinterpret_cast<uint2*>(Wf + (size_t)(Cout + ti * 16 + r) * Cin + tj * 16 + 4 * g) = pk;
    }
    return;
  }
  b -= nG;
  if (b < nB) {   // ---- bias b[i] = sum_k k3[k] W[k][i], one wave per i
    const int i = b * 4 + wid;
    if (i >= Cin) return;
    float acc = 0.f;
    for (int kk = lane; kk < Cout; kk += 64) {
      const uint32_t u = W[(size_t)kk * Cin + i];
      acc = __builtin_fmaf(k3[kk], unpack2<DT>(u).x, acc);
    }
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
    if (lane == 0) bias[i] = acc;
    return;
  }
  b -= nB;   // ---- rows [0, Cout): k1 o W, one 16-B chunk per thread
  const int c = b * 256 + tid;
  const int cpr = Cin >> 3;
  if (c >= Cout * cpr) return;
  const int row = c / cpr;
  const float s1 = k1[row];
  const i32x4 v = *reinterpret_cast<const i32x4*>(W + (size_t)c * 8);
  i32x4 o;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const f32x2 f = unpack2<DT>((uint32_t)v[q]);
    o[q] = (int)pack2<DT>(f32x2{f.x * s1, f.y * s1});
  }
  *reinterpret_cast<i32x4*>(Wf + (size_t)c * 8) = o;
}

// B = W Gram (f32 [Cout][C]) for the decomposed tail-fold weight gradient: W 16-bit [Cout][C] (the
// weights the forward used), Gram f32 [C][C]. Thread: one row, 4 consecutive columns, j in order.
template <int DT>
__global__ __launch_bounds__(256) void fold_bgemm_kernel(const u16* __restrict__ W,
                                                         const float* __restrict__ gram, int Cout,
                                                         int C, float* __restrict__ B) {
  const int t = blockIdx.x * 256 + threadIdx.x;
  const int c4 = C >> 2;
  if (t >= Cout * c4) return;
  const int row = t / c4, n = (t - row * c4) * 4;
  const u16* w = W + (size_t)row * C;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  for (int j = 0; j < C; j += 2) {
    const f32x2 wv = unpack2<DT>(*reinterpret_cast<const uint32_t*>(w + j));
    acc += wv.x * *reinterpret_cast<const f32x4*>(gram + (size_t)j * C + n);
    acc += wv.y * *reinterpret_cast<const f32x4*>(gram + (size_t)(j + 1) * C + n);
  }
  *reinterpret_cast<f32x4*>(B + (size_t)row * C + n) = acc;
}

}  // namespace

// ================================================================= host launchers (C ABI)
static FastDiv make_div(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

struct ConvDesc {  // mirrors pytorch_distributed_amd/ops/ext.py ConvDesc
  int Nb, H, W, Cin, Cout, R, S, stride, pad, Ho, Wo;
};

template <int PASS, int DT, int BM, int BN, int ST>
static int launch(const ConvParams& p, dim3 grid, hipStream_t st) {
  if constexpr ((PASS == WGRAD_BNA || PASS == DGRAD_BNF || PASS == WGRAD_GRAM || PASS == FWD_TAIL) &&
                DT != DT_BF16 && DT != DT_F16) {
    return -1;
  } else {
    TRACKED_LAUNCH((conv_gemm_kernel<PASS, DT, BM, BN, ST>), grid, dim3(conv_nt<ST>()), 0, st, p);
    return (int)hipGetLastError();
  }
}

// Tile codes: bm < 0 selects the single-buffer (STAGES = 1) variant of tile |bm| x bn; bm > 1000
// the LDS-DMA 8-wave variant (STAGES = 3) of tile (bm - 1000) x bn (16-bit, no operand prologue).
// bm > 2000: the tap-reuse (HALO) variant of (bm - 2000) x bn for 3x3 stride-1 FWD / DGRAD.
static int tile_bm(int bm) { return bm > 2000 ? bm - 2000 : bm > 1000 ? bm - 1000 : (bm < 0 ? -bm : bm); }
static bool halo_ok(const ConvParams& p, int csz) {
  return p.R == 3 && p.S == 3 && p.stride == 1 && p.pad == 1 && p.W <= 63 && csz % 64 == 0 &&
         p.Ho == p.H && p.Wo == p.W;
}

template <int PASS>
static int dispatch(int dt, int bm, int bn, const ConvParams& p, dim3 grid, hipStream_t st) {
  if (bm > 2000) {
    if constexpr (PASS != WGRAD) {
      if (p.pro_sc != nullptr || !halo_ok(p, PASS == FWD ? p.Cin : p.Cout)) return -5;
#define TILE_CASE4(D, M_, N_)                                                   \
  if (dt == D && bm - 2000 == M_ && bn == N_) return launch<PASS, D, M_, N_, 4>(p, grid, st);
      TILE_CASE4(DT_BF16, 256, 128) TILE_CASE4(DT_BF16, 256, 64)
#ifndef CONV_DMA_ONLY
      TILE_CASE4(DT_F16, 256, 128) TILE_CASE4(DT_F16, 256, 64)
#endif
#undef TILE_CASE4
    }
    return -1;
  }
  if (bm > 1000) {
    if (p.pro_sc != nullptr) return -5;   // the operand prologue needs register staging
#define TILE_CASE3(D, M_, N_)                                                   \
  if (dt == D && bm - 1000 == M_ && bn == N_) return launch<PASS, D, M_, N_, 3>(p, grid, st);
    TILE_CASE3(DT_BF16, 256, 128) TILE_CASE3(DT_BF16, 128, 256) TILE_CASE3(DT_BF16, 128, 128)
    if constexpr (PASS == WGRAD) { TILE_CASE3(DT_BF16, 256, 256) }
#ifndef CONV_DMA_ONLY
    TILE_CASE3(DT_F16, 256, 128) TILE_CASE3(DT_F16, 128, 256) TILE_CASE3(DT_F16, 128, 128)
    if constexpr (PASS == WGRAD) { TILE_CASE3(DT_F16, 256, 256) }
#endif
#undef TILE_CASE3
    return -1;
  }
#ifndef CONV_DMA_ONLY   // experiment builds (tools/dma_ab.py): the LDS-DMA kernels only
  if (bm < 0) {
#define TILE_CASE1(D, M_, N_)                                                   \
  if (dt == D && -bm == M_ && bn == N_) return launch<PASS, D, M_, N_, 1>(p, grid, st);
    TILE_CASE1(DT_BF16, 128, 128) TILE_CASE1(DT_BF16, 128, 64) TILE_CASE1(DT_BF16, 64, 128)
    // 256-wide tiles only where they measured faster (profiles/convbench_r1_v6.txt): wgrad 256x128
    // (3x3 layers 3-4; the dgrad 128x256 tile never beat 128x128 in the step and is not built)
    if constexpr (PASS == WGRAD) { TILE_CASE1(DT_BF16, 256, 128) TILE_CASE1(DT_F16, 256, 128) }
    // 256x64 forward (the N = 64 stem: K = 256 is 4 k-tiles, so a block's life is mostly its load
    // -> MFMA -> epilogue latency chain; twice the rows per chain)
    if constexpr (PASS == FWD) { TILE_CASE1(DT_BF16, 256, 64) TILE_CASE1(DT_F16, 256, 64) }
    TILE_CASE1(DT_F16, 128, 128) TILE_CASE1(DT_F16, 128, 64) TILE_CASE1(DT_F16, 64, 128)
    TILE_CASE1(DT_F32, 128, 128) TILE_CASE1(DT_F32, 128, 64) TILE_CASE1(DT_F32, 64, 128)
    // the split-f32 path stages hi + lo tiles: single-stage only (LDS)
    TILE_CASE1(DT_F32S, 128, 128) TILE_CASE1(DT_F32S, 128, 64) TILE_CASE1(DT_F32S, 64, 128)
    TILE_CASE1(DT_F32S, 64, 64)
#undef TILE_CASE1
    return -1;
  }
#define TILE_CASE(D, M_, N_)                                                    \
  if (dt == D && bm == M_ && bn == N_) return launch<PASS, D, M_, N_, 2>(p, grid, st);
  TILE_CASE(DT_BF16, 128, 128) TILE_CASE(DT_BF16, 128, 64) TILE_CASE(DT_BF16, 64, 128)
  TILE_CASE(DT_BF16, 64, 64)
  TILE_CASE(DT_F16, 128, 128) TILE_CASE(DT_F16, 128, 64) TILE_CASE(DT_F16, 64, 128)
  TILE_CASE(DT_F16, 64, 64)
  TILE_CASE(DT_F32, 128, 128) TILE_CASE(DT_F32, 128, 64) TILE_CASE(DT_F32, 64, 128)
  TILE_CASE(DT_F32, 64, 64)
#undef TILE_CASE
#endif
  return -1;
}

// the kernels address operands with 32-bit buffer offsets (range-checked, OOB = 0x80000000)
static bool fits32(long long a, long long b, long long c, int dt) {
  const long long lim = 0x7fffffffll, es = (dt == DT_F32 || dt == DT_F32S) ? 4 : 2;
  return a * es < lim && b * es < lim && c * 4 < lim;
}

static void fill_geom(ConvParams& p, const ConvDesc& d) {
  p.Nb = d.Nb; p.H = d.H; p.W = d.W; p.Cin = d.Cin; p.Cout = d.Cout;
  p.R = d.R; p.S = d.S; p.stride = d.stride; p.pad = d.pad; p.Ho = d.Ho; p.Wo = d.Wo;
  int l = 0;
  while ((1 << l) < d.Cin) ++l;
  p.log2Cin = l;
  int lo = 0;
  while ((1 << lo) < d.Cout) ++lo;
  p.log2Cout = (1 << lo) == d.Cout ? lo : -1;
  p.dHoWo = make_div(d.Ho * d.Wo);
  p.dWo = make_div(d.Wo);
  p.dS = make_div(d.S);
}

extern "C" {

// Y[M=Nb*Ho*Wo][Cout] = conv(X, W). W: [Cout][Kpad] 16-bit. stats: [ceil(M/bm)][3][Cout] shifted
// partials or null.
int pda_conv_fwd(const ConvDesc* d, const void* x, const void* w, int Kpad, void* y, int out_f32,
                 int out_pitch, const float* bias, float* stats, int relu, const float* pro_sc,
                 const float* pro_sh, int dt, int bm, int bn, hipStream_t st) {
  if (!fits32((long long)d->Nb * d->H * d->W * d->Cin, (long long)d->Cout * Kpad,
              (long long)d->Nb * d->Ho * d->Wo * d->Cout, dt) || d->R * d->S > 64)
    return -4;
  ConvParams p{};
  fill_geom(p, *d);
  p.pro_sc = pro_sc; p.pro_sh = pro_sh;
  p.a = x; p.b = w; p.out = y; p.stats = stats; p.bias = bias;
  p.M = d->Nb * d->Ho * d->Wo; p.N = d->Cout; p.Kpad = Kpad; p.K = Kpad;
  p.out_f32 = out_f32; p.relu = relu; p.out_pitch = out_pitch > 0 ? out_pitch : d->Cout;
  if (bm > 1000 && (d->Cin < 64 || (d->Cin & (d->Cin - 1)))) return -5;   // DMA: one tap per k-tile
  const int abm = tile_bm(bm);
  const int tiles = ((p.M + abm - 1) / abm) * ((p.N + bn - 1) / bn);
  return dispatch<FWD>(dt, bm, bn, p, dim3(tiles, 1), st);
}

// FWD_TAIL (see the Pass enum): Y = conv(a, W) of a 1x1 stride-1 conv whose input
// a = relu(y3 * sc + sh + r) (mode 1, r = res) or relu(y3 * sc + sh + res * sc2 + sh2) (mode 2) is
// formed while staging; a is written to a_out (and its ReLU bitmask to mask, mode 1, nullable) by
// the first N-tile's blocks. Register-staged single-stage tiles (-128, 64) / (-128, 128).
int pda_conv_fwd_tail(const ConvDesc* d, const void* y3, const void* w, int Kpad, void* y,
                      float* stats, const float* sc, const float* sh, const void* res,
                      const float* sc2, const float* sh2, void* a_out, void* mask, int mode, int dt,
                      int bm, int bn, hipStream_t st) {
  if (dt != DT_BF16 && dt != DT_F16) return -1;
  if (d->R != 1 || d->S != 1 || d->stride != 1 || d->pad != 0 || (d->Cin % 64) || Kpad != d->Cin ||
      !sc || !sh || !res || !a_out || (mode != 1 && mode != 2) || (mode == 2 && (!sc2 || !sh2)))
    return -2;
  if (!fits32((long long)d->Nb * d->H * d->W * d->Cin, (long long)d->Cout * Kpad,
              (long long)d->Nb * d->Ho * d->Wo * d->Cout, dt))
    return -4;
  ConvParams p{};
  fill_geom(p, *d);
  p.pro_sc = sc; p.pro_sh = sh;
  p.pro_res = res; p.pro_sc2 = sc2; p.pro_sh2 = sh2; p.pro_out = a_out;
  p.pro_mask = (uint8_t*)mask; p.pro_mode = mode;
  p.a = y3; p.b = w; p.out = y; p.stats = stats; p.bias = nullptr;
  p.M = d->Nb * d->Ho * d->Wo; p.N = d->Cout; p.Kpad = Kpad; p.K = Kpad;
  p.out_f32 = 0; p.relu = 0; p.out_pitch = d->Cout;
  { const char* rv = pda_reverse_env(); p.rev = (rv && strstr(rv, "fwd_tail")) ? 1 : 0; }
  const int tiles = ((p.M + 127) / 128) * ((p.N + bn - 1) / bn);
#define TAIL_CASE(D, N_) \
  if (dt == D && bm == -128 && bn == N_) return launch<FWD_TAIL, D, 128, N_, 1>(p, dim3(tiles, 1), st);
#ifndef CONV_DMA_ONLY
  TAIL_CASE(DT_BF16, 64) TAIL_CASE(DT_BF16, 128) TAIL_CASE(DT_F16, 64) TAIL_CASE(DT_F16, 128)
#endif
#undef TAIL_CASE
  return -1;
}

// dX[Nb,H,W,Cin] = conv_transpose(dY, W). Every dX element is written (zeros where no tap lands).
struct BnEpi {  // mirrors ops/ext.py BnEpi
  int mode, nq;
  const void* y; const float* sc; const float* sh;
  const void* y2; const float* sc2; const float* sh2;
  const void* g2; float* part;
  const void* mask;
};

static int dgrad_params(ConvParams& p, const ConvDesc* d, const void* dy, const void* w, void* dx,
                        const BnEpi* epi) {
  fill_geom(p, *d);
  p.a = dy; p.b = w; p.out = dx;
  p.emode = -1;
  if (epi) {
    p.emode = epi->mode; p.enq = epi->nq;
    p.ey = epi->y; p.esc = epi->sc; p.esh = epi->sh;
    p.ey2 = epi->y2; p.esc2 = epi->sc2; p.esh2 = epi->sh2;
    p.eg2 = epi->g2; p.epart = epi->part;
    p.emask = (const uint8_t*)epi->mask;
  }
  p.N = d->Cin; p.out_pitch = d->Cin;
  const int sd = d->stride;
  if (sd != 1 && sd != 2) return -2;
  if ((d->H % sd) || (d->W % sd) || (d->Cout % 64)) return -3;
  p.Hc = d->H / sd; p.Wc = d->W / sd;
  p.dHcWc = make_div(p.Hc * p.Wc);
  p.dWc = make_div(p.Wc);
  p.M = d->Nb * p.Hc * p.Wc;
  const int ncls = sd * sd;
  for (int c = 0; c < 4; ++c) {
    p.ntaps[c] = 0;
    if (c >= ncls) continue;
    const int ph = (sd == 2) ? (c >> 1) : 0, pw = (sd == 2) ? (c & 1) : 0;
    for (int r = 0; r < d->R; ++r) {
      if (((ph + d->pad - r) % sd + sd) % sd) continue;
      for (int s = 0; s < d->S; ++s) {
        if (((pw + d->pad - s) % sd + sd) % sd) continue;
        if (p.ntaps[c] < 9) {
          p.tdy[c][p.ntaps[c]] = (ph + d->pad - r) / sd;
          p.tdx[c][p.ntaps[c]] = (pw + d->pad - s) / sd;
          p.taps[c][p.ntaps[c]++] = r * d->S + s;
        }
      }
    }
  }
  p.K = 0;
  return 0;
}

int pda_conv_dgrad(const ConvDesc* d, const void* dy, const void* w, void* dx, const BnEpi* epi,
                   int dt, int bm, int bn, hipStream_t st) {
  if (!fits32((long long)d->Nb * d->Ho * d->Wo * d->Cout, (long long)d->Cout * d->R * d->S * d->Cin,
              (long long)d->Nb * d->H * d->W * d->Cin, dt))
    return -4;
  ConvParams p{};
  const int rc = dgrad_params(p, d, dy, w, dx, epi);
  if (rc) return rc;
  const int abm = tile_bm(bm);
  const int tiles = ((p.M + abm - 1) / abm) * ((p.N + bn - 1) / bn);
  return dispatch<DGRAD>(dt, bm, bn, p, dim3(tiles, d->stride * d->stride), st);
}

// DGRAD of a 1x1 conv whose dY = k1*dz + k2*y + k3 is folded (see DGRAD_BNF): dz [Nb,Ho,Wo,Cout];
// wf = [k1 o W ; G] ([Cout + Cin][Cin], pda_bn_fold); xa [Nb,H,W,Cin] the Gram operand (the conv's
// forward input; xa_sc / xa_sh: its BN+ReLU prologue, or null); dbias [Cin] f32. Register-staged
// tiles (-128, 64), (-128, 128), (64, 64), (64, 128); -1 otherwise.
int pda_conv_dgrad_bnf(const ConvDesc* d, const void* dz, const void* wf, void* dx, const BnEpi* epi,
                       const void* xa, const float* xa_sc, const float* xa_sh, const float* dbias,
                       int dt, int bm, int bn, hipStream_t st) {
  if (dt != DT_BF16 && dt != DT_F16) return -1;
  const int xa_c = d->Cin;
  if (d->R != 1 || d->S != 1 || d->pad != 0 || (d->Cin % 64) || !xa || !dbias) return -2;
  if (!fits32((long long)d->Nb * d->Ho * d->Wo * d->Cout, (long long)(d->Cout + d->Cin) * d->Cin,
              (long long)d->Nb * d->H * d->W * d->Cin, dt))
    return -4;
  ConvParams p{};
  const int rc = dgrad_params(p, d, dz, wf, dx, epi);
  if (rc) return rc;
  p.xa = xa; p.xa_sc = xa_sc; p.xa_sh = xa_sh; p.dbias = dbias; p.xa_c = xa_c;
  { const char* rv = pda_reverse_env(); p.rev = (rv && strstr(rv, "bnf")) ? 1 : 0; }
  const int abm = tile_bm(bm);
  const dim3 grid(((p.M + abm - 1) / abm) * ((p.N + bn - 1) / bn), d->stride * d->stride);
#define BNF_CASE(D, M_, N_, S_) \
  if (dt == D && bm == (S_ == 1 ? -M_ : M_) && bn == N_) return launch<DGRAD_BNF, D, M_, N_, S_>(p, grid, st);
#ifndef CONV_DMA_ONLY
  BNF_CASE(DT_BF16, 128, 64, 1) BNF_CASE(DT_BF16, 128, 128, 1) BNF_CASE(DT_BF16, 64, 64, 2)
  BNF_CASE(DT_BF16, 64, 128, 2)
  BNF_CASE(DT_F16, 128, 64, 1) BNF_CASE(DT_F16, 128, 128, 1) BNF_CASE(DT_F16, 64, 64, 2)
  BNF_CASE(DT_F16, 64, 128, 2)
#endif
#undef BNF_CASE
  return -1;
}

// Wf = [k1 o W ; W^T diag(k2) W] and b = W^T k3 of a 1x1 conv (W [Cout][Cin] 16-bit, k = [k1;k2;k3]
// 3 x Cout f32): the operands of pda_conv_dgrad_bnf. Cout, Cin multiples of 64.
int pda_bn_fold(const void* w, const float* k, int Cout, int Cin, void* wf, float* bias, int dt,
                hipStream_t st) {
  if ((Cout % 64) || (Cin % 64) || Cin > 4096) return -2;
  const int nG = (Cin / 16) * (Cin / 16), nB = Cin / 4, nR = (Cout * (Cin / 8) + 255) / 256;
  const dim3 grid(nG + nB + nR);
  if (dt == DT_BF16)
    TRACKED_LAUNCH(bn_fold_kernel<DT_BF16>, grid, dim3(256), 0, st, (const u16*)w, k, Cout, Cin,
                       (u16*)wf, bias, nG, nB);
  else if (dt == DT_F16)
    TRACKED_LAUNCH(bn_fold_kernel<DT_F16>, grid, dim3(256), 0, st, (const u16*)w, k, Cout, Cin,
                       (u16*)wf, bias, nG, nB);
  else
    return -1;
  return (int)hipGetLastError();
}

// As pda_conv_wgrad with dY formed while staging from the BatchNorm backward: dY = k1*dz + k2*y + k3
// (per output channel; the stem: Cout 64). 16-bit, 64x128 tiles only (wider ones spill); -1 otherwise.
int pda_conv_wgrad_bna(const ConvDesc* d, const void* dz, const void* y, const float* k1,
                       const float* k2, const float* k3, const void* x, float* slab, int splits,
                       int k_chunk, const float* pro_sc, const float* pro_sh, int dt, int bm, int bn,
                       hipStream_t st) {
  if (dt != DT_BF16 && dt != DT_F16) return -1;
  if (!fits32((long long)d->Nb * d->Ho * d->Wo * d->Cout, (long long)d->Nb * d->H * d->W * d->Cin,
              (long long)splits * d->Cout * d->R * d->S * d->Cin, dt) || (d->Cout % 8))
    return -4;
  ConvParams p{};
  fill_geom(p, *d);
  p.pro_sc = pro_sc; p.pro_sh = pro_sh;
  p.a = dz; p.a2 = y; p.ak1 = k1; p.ak2 = k2; p.ak3 = k3;
  p.b = x; p.out = slab;
  p.M = d->Cout; p.N = d->R * d->S * d->Cin;
  p.K = d->Nb * d->Ho * d->Wo;
  p.k_chunk = k_chunk;
  const int abm = bm < 0 ? -bm : bm;
  const dim3 grid(((p.M + abm - 1) / abm) * ((p.N + bn - 1) / bn), splits);
#define BNA_CASE(D, M_, N_, S_) \
  if (dt == D && bm == (S_ == 1 ? -M_ : M_) && bn == N_) return launch<WGRAD_BNA, D, M_, N_, S_>(p, grid, st);
#ifndef CONV_DMA_ONLY
  BNA_CASE(DT_BF16, 64, 128, 1) BNA_CASE(DT_BF16, 64, 128, 2) BNA_CASE(DT_BF16, 64, 256, 1)
  BNA_CASE(DT_F16, 64, 128, 1) BNA_CASE(DT_F16, 64, 128, 2) BNA_CASE(DT_F16, 64, 256, 1)
  // the bottleneck conv3 weight gradients of the consumer-side tail fold (DGRAD_BNF)
  BNA_CASE(DT_BF16, 128, 128, 1) BNA_CASE(DT_BF16, 128, 128, 2) BNA_CASE(DT_BF16, 128, 64, 1)
  BNA_CASE(DT_F16, 128, 128, 1) BNA_CASE(DT_F16, 128, 128, 2) BNA_CASE(DT_F16, 128, 64, 1)
#endif
#undef BNA_CASE
  return -1;
}

// Gram = a^T a and s = sum_p a_p of a = relu(sc*y + sh) (y [Nb,H,W,C] 16-bit; WGRAD_GRAM): slab
// [splits][C + 1][C] -- per split the partial Gram, then the partial column sums as row C (one
// split-K reduce gives both). Tiles (64, 64) two-stage, (-128, 128), (-128, 64); -1 otherwise.
int pda_conv_wgrad_gram(const ConvDesc* d, const void* y, const float* sc, const float* sh,
                        float* slab, int splits, int k_chunk, int dt, int bm, int bn, hipStream_t st) {
  if (dt != DT_BF16 && dt != DT_F16) return -1;
  if (d->R != 1 || d->S != 1 || d->stride != 1 || d->pad != 0 || d->Cin != d->Cout || (d->Cin % 8))
    return -2;
  if (!fits32((long long)d->Nb * d->H * d->W * d->Cin, 1, (long long)splits * d->Cin * (d->Cin + 1), dt))
    return -4;
  ConvParams p{};
  fill_geom(p, *d);
  p.pro_sc = sc; p.pro_sh = sh;
  p.a = y; p.ak1 = sc; p.ak3 = sh;
  p.b = y; p.out = slab;
  p.M = d->Cout; p.N = d->Cin;
  p.K = d->Nb * d->Ho * d->Wo;
  p.k_chunk = k_chunk;
  const int abm = bm < 0 ? -bm : bm;
  const dim3 grid(((p.M + abm - 1) / abm) * ((p.N + bn - 1) / bn), splits);
#define GRAM_CASE(D, M_, N_, S_) \
  if (dt == D && bm == (S_ == 1 ? -M_ : M_) && bn == N_) return launch<WGRAD_GRAM, D, M_, N_, S_>(p, grid, st);
#ifndef CONV_DMA_ONLY
  GRAM_CASE(DT_BF16, 64, 64, 2) GRAM_CASE(DT_BF16, 128, 128, 1) GRAM_CASE(DT_BF16, 128, 64, 1)
  GRAM_CASE(DT_F16, 64, 64, 2) GRAM_CASE(DT_F16, 128, 128, 1) GRAM_CASE(DT_F16, 128, 64, 1)
#endif
#undef GRAM_CASE
  return -1;
}

// B = W Gram (f32 [Cout][C]); W 16-bit [Cout][C], Gram f32 [C][C]. C a multiple of 4.
int pda_fold_bgemm(const void* w, const float* gram, int Cout, int C, float* b, int dt, hipStream_t st) {
  if (C % 4) return -2;
  const dim3 grid((Cout * (C / 4) + 255) / 256);
  if (dt == DT_BF16)
    TRACKED_LAUNCH(fold_bgemm_kernel<DT_BF16>, grid, dim3(256), 0, st, (const u16*)w, gram, Cout, C, b);
  else if (dt == DT_F16)
    TRACKED_LAUNCH(fold_bgemm_kernel<DT_F16>, grid, dim3(256), 0, st, (const u16*)w, gram, Cout, C, b);
  else
    return -1;
  return (int)hipGetLastError();
}

// slab[splits][Cout][R*S*Cin] partial weight gradients (f32). k_chunk must be a multiple of 64.
int pda_conv_wgrad(const ConvDesc* d, const void* dy, const void* x, float* slab, int splits,
                   int k_chunk, const float* pro_sc, const float* pro_sh, int dt, int bm, int bn,
                   hipStream_t st) {
  if (!fits32((long long)d->Nb * d->Ho * d->Wo * d->Cout, (long long)d->Nb * d->H * d->W * d->Cin,
              (long long)splits * d->Cout * d->R * d->S * d->Cin, dt))
    return -4;
  ConvParams p{};
  fill_geom(p, *d);
  p.pro_sc = pro_sc; p.pro_sh = pro_sh;
  p.a = dy; p.b = x; p.out = slab;
  p.M = d->Cout; p.N = d->R * d->S * d->Cin;
  p.K = d->Nb * d->Ho * d->Wo;
  p.k_chunk = k_chunk;
  const int abm = tile_bm(bm);
  const int tiles = ((p.M + abm - 1) / abm) * ((p.N + bn - 1) / bn);
  return dispatch<WGRAD>(dt, bm, bn, p, dim3(tiles, splits), st);
}

// Host-side descriptor of one queued reduction (mirrors ops/ext.py RedDescC).
struct RedDescC {
  const float* slab; float* grad; const float* ck; const float* cB; const float* cs;
  int splits, M, N, cin_log2, cin_real, pitch, accumulate;
  float scale;
};

// n (<= 24) split-K reductions of pda_wgrad_reduce's kind, N % 4 == 0 each, in one launch.
int pda_wgrad_reduce_batch(const RedDescC* ds, int n, hipStream_t st) {
  if (n <= 0) return 0;
  if (n > RB_MAX) return -2;
  RedBatch b{};
  b.n = n;
  int blk = 0;
  for (int i = 0; i < n; ++i) {
    const RedDescC& c = ds[i];
    if (c.N % 4 || c.M <= 0 || c.splits <= 0) return -2;
    RedDesc& d = b.d[i];
    d.slab = c.slab; d.grad = c.grad; d.ck = c.ck; d.cB = c.cB; d.cs = c.cs;
    d.splits = c.splits; d.M = c.M; d.N = c.N; d.cin_log2 = c.cin_log2; d.cin_real = c.cin_real;
    d.pitch = c.pitch; d.accumulate = c.accumulate; d.scale = c.scale; d.blk0 = blk;
    blk += (c.M * c.N + 63) / 64;
  }
  TRACKED_LAUNCH(wgrad_reduce_batch_kernel, dim3(blk), dim3(256), 0, st, b);
  return (int)hipGetLastError();
}

int pda_wgrad_reduce(const float* slab, float* grad, int splits, int M, int N, int cin_pad_log2,
                     int cin_real, int dst_pitch, float scale, int accumulate, const float* ck,
                     const float* cB, const float* cs, hipStream_t st) {
  const int total = M * N;
  if ((N & 3) == 0) {
    int epb = 256;
    // >= 256 blocks (fewer, fatter blocks than the 1024 of round 4: the reductions run on the
    // second stream beside the main chain; -0.025 ms/step over 4 alternating pairs, ab_r5.md s.16)
    while (epb > 16 && total / epb < 256) epb >>= 1;
    const dim3 grid((total + epb - 1) / epb);
#define RED_CASE(E)                                                                              \
  if (epb == E) {                                                                               \
    TRACKED_LAUNCH(wgrad_reduce4_kernel<E>, grid, dim3(256), 0, st, slab, grad, splits, M, N, \
                       cin_pad_log2, cin_real, dst_pitch, scale, accumulate, ck, cB, cs);       \
    return (int)hipGetLastError();                                                              \
  }
    RED_CASE(256) RED_CASE(128) RED_CASE(64) RED_CASE(32) RED_CASE(16)
#undef RED_CASE
  }
  int blocks = (total + 255) / 256;
  if (blocks > 4096) blocks = 4096;
  TRACKED_LAUNCH(wgrad_reduce_kernel, dim3(blocks), dim3(256), 0, st, slab, grad, splits, M, N,
                     cin_pad_log2, cin_real, dst_pitch, scale, accumulate, ck, cB, cs);
  return (int)hipGetLastError();
}

}  // extern "C"
