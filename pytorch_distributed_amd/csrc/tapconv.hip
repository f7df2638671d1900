// 3x3 / stride 1 / pad 1, 64 -> 64 channel convolution forward on gfx950 with tap reuse: the
// ResNet-50 layer1 conv2 (56x56, three per step; reference model: torchvision resnet50 built in
// /root/reference/resnet_single_gpu.py:27-31). Optional fused BN+ReLU prologue on the input and
// shifted BN partials in the epilogue, as conv_gemm.hip's FWD pass.
//
// Why: the generic implicit-GEMM tile re-gathers every 3x3 tap of every pixel from L2 (K = 576:
// 9x the input through L2 -> LDS) and re-applies the BN+ReLU prologue once per tap; it runs this
// shape at 166 us isolated and 210-250 us in the step with the prologue (~400 TF/s), while the
// layer's MFMA work is ~37 us and its HBM traffic ~65 us at batch 400.
// Here an input slab of (8 + 2) rows x (W + 2) columns x 64 channels is staged into LDS ONCE per
// 8-row tile (BN+ReLU applied once, zero padding written explicitly) and the MFMA pixel operand
// (8 channels of one tap of one pixel = 16 contiguous bytes) is read straight from it. The whole
// 64 x 576 weight matrix stays in LDS for the persistent block.
//
// Block: 8 waves; wave w owns output rows 2(w >> 1), +1 of the tile (2W pixels = W / 8 fragments of
// 16) and output channels 32 (w & 1) .. +31 (two 16-channel fragments).
// MFMA 16x16x32: A = weights (rows = output channel), B = pixels, so a lane holds 4 consecutive
// channels of one pixel (8-byte stores). LDS layouts are XOR-swizzled by 16-byte chunk so the 16
// rows / pixels of one fragment read hit distinct bank quads.
// Statistics: per wave, shifted partials over its 2 rows (2W consecutive rows of M, shift = the
// first pixel) for its 32 channels; fixed reduction order (deterministic).
#include "common.h"

namespace {

constexpr int TC_NT = 512;           // 8 waves
constexpr int TC_TH = 8;             // output rows per tile
constexpr int TC_SR = TC_TH + 2;     // slab rows
constexpr int TC_C = 64;             // input = output channels
constexpr int TC_K = 576;            // 9 taps x 64 channels
constexpr int TC_KC = TC_K / 8;      // 16-byte chunks per weight row (72)

// weight row c: 72 chunks; chunk kc at position kc ^ ((c >> 1) & 7) (stays inside its 8-group)
__device__ __forceinline__ int tw_off(int c, int kc) { return c * (TC_K * 2) + ((kc ^ ((c >> 1) & 7)) << 4); }
// slab pixel (row, col): 8 chunks of 8 channels; chunk c8 at position c8 ^ (col & 7)
template <int SW>
__device__ __forceinline__ int ts_off(int row, int col, int c8) { return ((row * SW + col) * 8 + (c8 ^ (col & 7))) << 4; }

template <int DT, int PF, bool STATS, bool PRO>
__global__ __launch_bounds__(TC_NT, 1) void tapconv_fwd_kernel(
    const u16* __restrict__ x, const u16* __restrict__ w, u16* __restrict__ y,
    float* __restrict__ stats, const float* __restrict__ psc, const float* __restrict__ psh,
    int H, int tiles, int tiles_per_block) {
  constexpr int W = PF * 8;                      // 2 rows per wave = PF fragments of 16 pixels
  constexpr int SW = W + 2;                      // slab columns: input cols -1 .. W
  constexpr int NCH = TC_SR * SW * 8;            // 16-byte chunks in the slab
  constexpr int PT = (NCH + TC_NT - 1) / TC_NT;  // chunks per thread
  constexpr int LDS = TC_C * TC_K * 2 + NCH * 16 + 2 * TC_C * 4;
  static_assert(LDS <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) char smem[LDS];
  char* sw = smem;                               // weights, 72 KiB
  char* ss = smem + TC_C * TC_K * 2;             // input slab
  float* lsc = reinterpret_cast<float*>(ss + NCH * 16);   // prologue scale / shift [64] each

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int rp = wave >> 1, ch0 = (wave & 1) * 32;   // row pair, first output channel
  const int t0 = blockIdx.x * tiles_per_block;
  const int t1 = min(tiles, t0 + tiles_per_block);
  if (t0 >= t1) return;
  const int tpi = H / TC_TH;

  for (int i = tid; i < TC_C * TC_KC; i += TC_NT) {
    const int c = i / TC_KC, kc = i - c * TC_KC;
    *reinterpret_cast<i32x4*>(sw + tw_off(c, kc)) =
        *reinterpret_cast<const i32x4*>(w + (size_t)c * TC_K + kc * 8);
  }
  if constexpr (PRO) {
    if (tid < TC_C) {
      lsc[tid] = psc[tid];
      lsc[TC_C + tid] = psh[tid];
    }
  }
  __syncthreads();   // the prologue coefficients are read while staging

  i32x4 pre[PT];
  auto load_slab = [&](int t) {
    const int n = t / tpi, oy0 = (t - n * tpi) * TC_TH;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + i * TC_NT;
      const int pix = ch >> 3, c8 = ch & 7;
      const int row = pix / SW, col = pix - row * SW;
      const int iy = oy0 - 1 + row, ix = col - 1;
      i32x4 v = i32x4{0, 0, 0, 0};
      if (ch < NCH && iy >= 0 && iy < H && ix >= 0 && ix < W)
        v = *reinterpret_cast<const i32x4*>(x + (((size_t)n * H + iy) * W + ix) * TC_C + c8 * 8);
      pre[i] = v;
    }
  };
  auto store_slab = [&](int t) {
    const int n = t / tpi, oy0 = (t - n * tpi) * TC_TH;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + i * TC_NT;
      if (ch >= NCH) continue;
      const int pix = ch >> 3, c8 = ch & 7;
      const int row = pix / SW, col = pix - row * SW;
      i32x4 v = pre[i];
      if constexpr (PRO) {   // relu(x * sc + sh) inside the image; the padding stays 0
        const int iy = oy0 - 1 + row, ix = col - 1;
        if (iy >= 0 && iy < H && ix >= 0 && ix < W) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const int c = c8 * 8 + 2 * k;
            f32x2 f = unpack2<DT>((uint32_t)v[k]);
            f = f * f32x2{lsc[c], lsc[c + 1]} + f32x2{lsc[TC_C + c], lsc[TC_C + c + 1]};
            f = f32x2{fmaxf(f.x, 0.f), fmaxf(f.y, 0.f)};
            v[k] = (int)pack2<DT>(f);
          }
        }
      }
      *reinterpret_cast<i32x4*>(ss + ts_off<SW>(row, col, c8)) = v;
    }
  };
  load_slab(t0);

  // lane pixels of the wave's 2-row span: fragment p, pixel 16p + l16 -> (row in pair, col)
  int prow[PF], pcol[PF];
#pragma unroll
  for (int p = 0; p < PF; ++p) {
    const int j = 16 * p + l16;
    prow[p] = j >= W ? 1 : 0;
    pcol[p] = j - prow[p] * W;
  }

  for (int t = t0; t < t1; ++t) {
    __syncthreads();   // every wave is done reading the previous tile's slab
    store_slab(t);
    __syncthreads();
    if (t + 1 < t1) load_slab(t + 1);   // in flight under this tile's MFMAs

    f32x4 acc[PF][2];
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int f = 0; f < 2; ++f) acc[p][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
    for (int ks = 0; ks < TC_K / 32; ++ks) {
      s16x8 a[2];
#pragma unroll
      for (int f = 0; f < 2; ++f)
        a[f] = *reinterpret_cast<const s16x8*>(sw + tw_off(ch0 + 16 * f + l16, 4 * ks + q));
      // lane: tap ks >> 1, channels 32 (ks & 1) + 8q .. +7
      const int tap = ks >> 1, r = tap / 3, s = tap - 3 * r, c8 = (ks & 1) * 4 + q;
#pragma unroll
      for (int p = 0; p < PF; ++p) {
        const s16x8 b = *reinterpret_cast<const s16x8*>(
            ss + ts_off<SW>(2 * rp + prow[p] + r, pcol[p] + s, c8));
#pragma unroll
        for (int f = 0; f < 2; ++f) acc[p][f] = mfma16<DT>(a[f], b, acc[p][f]);
      }
    }

    // ---- epilogue: rounded stores + shifted statistics of the wave's 2 rows, 32 channels
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    const int n = t / tpi, oy = (t - n * tpi) * TC_TH + 2 * rp;
    u16* yb = y + (((size_t)n * H + oy) * W) * TC_C + ch0;   // pixel j of the pair at yb + j * 64
    float sh[2][4];
    if constexpr (STATS) {   // shift = the pair's first pixel, broadcast from lane 16q
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const f32x2 lo = unpack2<DT>(pack2<DT>(f32x2{acc[0][f][0], acc[0][f][1]}));
        const f32x2 hi = unpack2<DT>(pack2<DT>(f32x2{acc[0][f][2], acc[0][f][3]}));
        const float e[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
        for (int i = 0; i < 4; ++i) sh[f][i] = __shfl(e[i], lane & 48, 64);
      }
    }
    float v[16];   // [q0 | q1][f][i] of channel ch0 + 16f + 4q + i
#pragma unroll
    for (int j = 0; j < 16; ++j) v[j] = 0.f;
#pragma unroll
    for (int p = 0; p < PF; ++p)
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const uint32_t w0 = pack2<DT>(f32x2{acc[p][f][0], acc[p][f][1]});
        const uint32_t w1 = pack2<DT>(f32x2{acc[p][f][2], acc[p][f][3]});
        *reinterpret_cast<u32x2*>(yb + (size_t)(16 * p + l16) * TC_C + 16 * f + 4 * q) = u32x2{w0, w1};
        if constexpr (STATS) {
          const f32x2 lo = unpack2<DT>(w0), hi = unpack2<DT>(w1);
          const float e[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const float d = e[i] - sh[f][i];
            v[f * 4 + i] += d;
            v[8 + f * 4 + i] += d * d;
          }
        }
      }
    if constexpr (!STATS) continue;
    // halving butterfly over the 16 pixel lanes: lane l16 ends with entry l16
#pragma unroll
    for (int m = 8, c = 16; m >= 1; m >>= 1, c >>= 1) {
      const bool hi = (l16 & m) != 0;
#pragma unroll
      for (int j = 0; j < c / 2; ++j) {
        const float send = hi ? v[j] : v[j + c / 2];
        const float keep = hi ? v[j + c / 2] : v[j];
        v[j] = keep + __shfl_xor(send, m, 64);
      }
    }
    {
      float* base = stats + ((size_t)t * (TC_TH / 2) + rp) * 3 * TC_C + ch0;
      const int qs = l16 >> 3, f = (l16 >> 2) & 1, i = l16 & 3;
      base[qs * TC_C + 16 * f + 4 * q + i] = v[0];
      if (l16 == 0) {
#pragma unroll
        for (int f2 = 0; f2 < 2; ++f2)
          *reinterpret_cast<f32x4*>(base + 2 * TC_C + 16 * f2 + 4 * q) =
              f32x4{sh[f2][0], sh[f2][1], sh[f2][2], sh[f2][3]};
      }
    }
  }
}

template <int DT, int PF>
int launch_tapconv(const void* x, const void* w, void* y, float* stats, const float* sc,
                   const float* sh, int Nb, int H, int grid_cap, hipStream_t st) {
  constexpr int W = PF * 8;
  const int tiles = Nb * (H / TC_TH);
  const int cap = grid_cap > 0 ? grid_cap : 256;
  const int tpb = (tiles + cap - 1) / cap;
  const int grid = (tiles + tpb - 1) / tpb;
  const u16* xx = (const u16*)x;
  const u16* ww = (const u16*)w;
  u16* yy = (u16*)y;
  if (stats && sc)
    hipLaunchKernelGGL((tapconv_fwd_kernel<DT, PF, true, true>), dim3(grid), dim3(TC_NT), 0, st,
                       xx, ww, yy, stats, sc, sh, H, tiles, tpb);
  else if (stats)
    hipLaunchKernelGGL((tapconv_fwd_kernel<DT, PF, true, false>), dim3(grid), dim3(TC_NT), 0, st,
                       xx, ww, yy, stats, sc, sh, H, tiles, tpb);
  else if (sc)
    hipLaunchKernelGGL((tapconv_fwd_kernel<DT, PF, false, true>), dim3(grid), dim3(TC_NT), 0, st,
                       xx, ww, yy, stats, sc, sh, H, tiles, tpb);
  else
    hipLaunchKernelGGL((tapconv_fwd_kernel<DT, PF, false, false>), dim3(grid), dim3(TC_NT), 0, st,
                       xx, ww, yy, stats, sc, sh, H, tiles, tpb);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace

// y [Nb][H][W][64] = conv3x3/1/1 (x [Nb][H][W][64], w [64][576] OHWI), 16-bit; sc/sh (nullable):
// x is PRE-BatchNorm and the conv consumes relu(x*sc + sh); stats (nullable) [Nb*H/2][3][64]
// shifted partials per output-row pair (2W rows of M). Requires H % 8 == 0, W % 8 == 0,
// 8 <= W <= 64; returns -1 otherwise.
extern "C" int pda_tapconv_fwd(const void* x, const void* w, void* y, float* stats, const float* sc,
                               const float* sh, int Nb, int H, int W, int dt, int grid_cap,
                               hipStream_t st) {
  if (Nb <= 0 || H <= 0 || H % TC_TH || W % 8 || W < 8 || W > 64 || (dt != DT_BF16 && dt != DT_F16))
    return -1;
  if ((sc == nullptr) != (sh == nullptr)) return -1;
#define TC_CASE(PFV)                                                                                \
  case PFV:                                                                                         \
    return dt == DT_BF16 ? launch_tapconv<DT_BF16, PFV>(x, w, y, stats, sc, sh, Nb, H, grid_cap, st) \
                         : launch_tapconv<DT_F16, PFV>(x, w, y, stats, sc, sh, Nb, H, grid_cap, st);
  switch (W / 8) {
    TC_CASE(1) TC_CASE(2) TC_CASE(3) TC_CASE(4)
    TC_CASE(5) TC_CASE(6) TC_CASE(7) TC_CASE(8)
  }
#undef TC_CASE
  return -1;
}
