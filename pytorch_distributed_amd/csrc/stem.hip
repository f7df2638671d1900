// Stem forward of ResNet-50 on gfx950: the 7x7/2 conv as a 4x4/1 conv (pad 2 top/left) over the
// 2x2 space-to-depth image (16 channels), with the BatchNorm forward statistics in the epilogue.
// Reference behaviour: torchvision resnet50 conv1 + bn1 (/root/reference/resnet_single_gpu.py:27-31
// builds the model; the stem is its first layer).
//
// Why a dedicated kernel: the generic implicit-GEMM tile gathers every 4x4 tap of a pixel from
// L2 (K = 256 is 16 taps x 16 channels, a 16x re-read of a 160 MB input) and its K loop is only 8
// steps deep, so it runs at ~350 TF/s and ~1.7 TB/s (455 us at batch 400, profiles/ab_r4.md s3),
// far from both bounds (~66 us of MFMA, ~170 us of HBM: 642 MB written, 160 MB read).
// Here the input is staged ONCE per tile into LDS as a zero-padded slab of (4 + 3) rows x (W + 3)
// columns, and the MFMA B operand (8 channels of one tap of one pixel = 16 contiguous bytes) is
// read from the slab directly: tap reuse without an im2col. Weights (64 x 256) stay in LDS for
// the whole persistent block.
//
// Tile = 4 output rows x W columns of one image (wave w owns row w), 64 output channels.
// MFMA 16x16x32: A = weights (rows = output channel), B = pixels (cols = pixel), so each lane
// holds 4 consecutive channels of one pixel: 8-byte stores, and one store instruction writes
// 16 pixels x 32 contiguous bytes.
// Statistics: shifted partials (sum(y - s), sum((y - s)^2), s) of the stored (rounded) values per
// output ROW (W consecutive rows of M; s = the row's first pixel), the format conv_gemm.hip's FWD
// epilogue writes and bn.hip bn_stats_kernel<0> finalizes. Each wave reduces its own row (a
// halving butterfly over its lanes), so the tile loop has no barrier besides the slab's.
// Fixed reduction order: deterministic.
#include "common.h"

#include <type_traits>

namespace {

constexpr int ST_NT = 256;              // 4 waves
constexpr int ST_TH = 4;                // output rows per tile (one per wave)
constexpr int ST_SR = ST_TH + 3;        // slab rows (4x4 taps)
constexpr int ST_C = 64;                // output channels
constexpr int ST_K = 256;               // 16 taps x 16 channels
constexpr int ST_PG = 4;                // pixel fragments per accumulator pass (PF <= 2 * ST_PG)

// weights in LDS: row c (512 B) holds 32 chunks of 8 k; chunk kc of row c lives at position
// kc ^ (c & 31), so the 16 rows of one A-fragment read hit 16 different bank quads
__device__ __forceinline__ int w_off(int c, int kc) { return c * 512 + ((kc ^ (c & 31)) << 4); }

template <int DT, int PF, bool STATS>
__global__ __launch_bounds__(ST_NT, 2) void stem_fwd_kernel(
    const u16* __restrict__ x, const u16* __restrict__ w, u16* __restrict__ y,
    float* __restrict__ stats, int H, int tiles, int tiles_per_block) {
  constexpr int W = PF * 16;
  constexpr int SW = W + 3;                       // slab columns: input cols -2 .. W
  constexpr int SLAB = ST_SR * SW * 32;           // bytes: 16 channels x 2 B per pixel
  constexpr int NCH = ST_SR * SW * 2;             // 16-byte chunks in the slab
  constexpr int PT = (NCH + ST_NT - 1) / ST_NT;   // chunks per thread
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* sw = smem;                                // weights, 32 KiB
  char* ss = smem + ST_C * 512;                   // input slab

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int l16 = lane & 15, q = lane >> 4;
  const int t0 = blockIdx.x * tiles_per_block;
  const int t1 = min(tiles, t0 + tiles_per_block);
  if (t0 >= t1) return;
  const int tpi = H / ST_TH;                      // tiles per image

  // weights -> LDS (64 x 256 x 2 B = 2048 chunks, 8 per thread)
#pragma unroll
  for (int i = 0; i < ST_C * ST_K / 8 / ST_NT; ++i) {
    const int ch = tid + i * ST_NT, c = ch >> 5, kc = ch & 31;
    *reinterpret_cast<i32x4*>(sw + w_off(c, kc)) =
        *reinterpret_cast<const i32x4*>(w + (size_t)c * ST_K + kc * 8);
  }

  i32x4 pre[PT];
  auto load_slab = [&](int t) {
    const int n = t / tpi, oy0 = (t - n * tpi) * ST_TH;
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + i * ST_NT;
      const int row = ch / (SW * 2), rem = ch - row * (SW * 2);
      const int col = rem >> 1, half = rem & 1;
      const int iy = oy0 - 2 + row, ix = col - 2;
      i32x4 v = i32x4{0, 0, 0, 0};
      if (ch < NCH && iy >= 0 && iy < H && ix >= 0 && ix < W)
        v = *reinterpret_cast<const i32x4*>(x + (((size_t)n * H + iy) * W + ix) * 16 + half * 8);
      pre[i] = v;
    }
  };
  load_slab(t0);

  for (int t = t0; t < t1; ++t) {
    __syncthreads();   // every wave is done reading the previous tile's slab (and the weights landed)
#pragma unroll
    for (int i = 0; i < PT; ++i) {
      const int ch = tid + i * ST_NT;
      if (ch < NCH) *reinterpret_cast<i32x4*>(ss + ch * 16) = pre[i];
    }
    __syncthreads();
    if (t + 1 < t1) load_slab(t + 1);   // in flight under this tile's MFMAs

    const int n = t / tpi, oy = (t - n * tpi) * ST_TH + wave;
    u16* yrow = y + (((size_t)n * H + oy) * W) * ST_C;
    float v[32];   // statistics: [q0 | q1][f][i] of channel 16f + 4q + i
#pragma unroll
    for (int j = 0; j < 32; ++j) v[j] = 0.f;
    float sh[4][4];
    // the row's PF pixel fragments in passes of at most PG (bounded accumulator registers); the
    // weight fragments are re-read from LDS per pass
    auto pass = [&](auto p0c, auto npc) {
      constexpr int P0 = decltype(p0c)::value, NP = decltype(npc)::value;
      f32x4 acc[NP][4];
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int f = 0; f < 4; ++f) acc[p][f] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 2
      for (int ks = 0; ks < ST_K / 32; ++ks) {
        s16x8 a[4];
#pragma unroll
        for (int f = 0; f < 4; ++f)
          a[f] = *reinterpret_cast<const s16x8*>(sw + w_off(16 * f + l16, 4 * ks + q));
        // lane: tap 2ks + (q >> 1), channels 8 (q & 1) .. +7 of pixel 16p + l16 of row `wave`
        const int tap = 2 * ks + (q >> 1), r = tap >> 2, s = tap & 3;
        const char* bp = ss + (((wave + r) * SW + 16 * P0 + l16 + s) * 2 + (q & 1)) * 16;
#pragma unroll
        for (int p = 0; p < NP; ++p) {
          const s16x8 b = *reinterpret_cast<const s16x8*>(bp + p * 16 * 32);
#pragma unroll
          for (int f = 0; f < 4; ++f) acc[p][f] = mfma16<DT>(a[f], b, acc[p][f]);
        }
      }
      // ---- epilogue: rounded stores + shifted statistics (shift = the tile's first pixel
      // (oy0, 0), published by wave 0 in the first pass before any wave folds its pixels in)
      typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
      if constexpr (STATS && P0 == 0) {   // shift = the wave's first pixel (its row's x = 0)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const f32x2 lo = unpack2<DT>(pack2<DT>(f32x2{acc[0][f][0], acc[0][f][1]}));
          const f32x2 hi = unpack2<DT>(pack2<DT>(f32x2{acc[0][f][2], acc[0][f][3]}));
          const float e[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
          for (int i = 0; i < 4; ++i) sh[f][i] = __shfl(e[i], lane & 48, 64);
        }
      }
#pragma unroll
      for (int p = 0; p < NP; ++p)
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          const uint32_t w0 = pack2<DT>(f32x2{acc[p][f][0], acc[p][f][1]});
          const uint32_t w1 = pack2<DT>(f32x2{acc[p][f][2], acc[p][f][3]});
          *reinterpret_cast<u32x2*>(yrow + (size_t)(16 * (P0 + p) + l16) * ST_C + 16 * f + 4 * q) =
              u32x2{w0, w1};
          if constexpr (STATS) {
            const f32x2 lo = unpack2<DT>(w0), hi = unpack2<DT>(w1);
            const float e[4] = {lo.x, lo.y, hi.x, hi.y};
#pragma unroll
            for (int i = 0; i < 4; ++i) {
              const float d = e[i] - sh[f][i];
              v[f * 4 + i] += d;
              v[16 + f * 4 + i] += d * d;
            }
          }
        }
    };
    using I0 = std::integral_constant<int, 0>;
    if constexpr (PF <= ST_PG) {
      pass(I0{}, std::integral_constant<int, PF>{});
    } else {
      pass(I0{}, std::integral_constant<int, ST_PG>{});
      pass(std::integral_constant<int, ST_PG>{}, std::integral_constant<int, PF - ST_PG>{});
    }
    if constexpr (!STATS) continue;
    // halving butterfly over the 16 pixel lanes of each channel group: after the xor-8/4/2/1
    // steps lane l16 holds the full sums of entries 2*l16 and 2*l16 + 1
#pragma unroll
    for (int m = 8, c = 32; m >= 1; m >>= 1, c >>= 1) {
      const bool hi = (l16 & m) != 0;
#pragma unroll
      for (int j = 0; j < c / 2; ++j) {
        const float send = hi ? v[j] : v[j + c / 2];
        const float keep = hi ? v[j + c / 2] : v[j];
        v[j] = keep + __shfl_xor(send, m, 64);
      }
    }
    {
      float* base = stats + ((size_t)t * ST_TH + wave) * 3 * ST_C;
      const int qs = l16 >> 3, f = (l16 >> 1) & 3, i0 = (l16 & 1) * 2;
      float* dst = base + qs * ST_C + 16 * f + 4 * q + i0;
      dst[0] = v[0];
      dst[1] = v[1];
      if (l16 == 0) {
#pragma unroll
        for (int f2 = 0; f2 < 4; ++f2)
          *reinterpret_cast<f32x4*>(base + 2 * ST_C + 16 * f2 + 4 * q) =
              f32x4{sh[f2][0], sh[f2][1], sh[f2][2], sh[f2][3]};
      }
    }
  }
}

template <int DT, int PF>
int launch_stem(const void* x, const void* w, void* y, float* stats, int Nb, int H, int grid_cap,
                hipStream_t st) {
  constexpr int W = PF * 16;
  const size_t lds = ST_C * 512 + (size_t)(ST_TH + 3) * (W + 3) * 32;
  const int tiles = Nb * (H / ST_TH);
  const int cap = grid_cap > 0 ? grid_cap : 1024;   // tools/stem_bench.py: 512-1024 best
  const int tpb = (tiles + cap - 1) / cap;
  const int grid = (tiles + tpb - 1) / tpb;
  if (stats)
    TRACKED_LAUNCH((stem_fwd_kernel<DT, PF, true>), dim3(grid), dim3(ST_NT), lds, st,
                       (const u16*)x, (const u16*)w, (u16*)y, stats, H, tiles, tpb);
  else
    TRACKED_LAUNCH((stem_fwd_kernel<DT, PF, false>), dim3(grid), dim3(ST_NT), lds, st,
                       (const u16*)x, (const u16*)w, (u16*)y, stats, H, tiles, tpb);
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // namespace

// y [Nb][H][W][64] = conv4x4/1 (pad 2 top/left) of x [Nb][H][W][16] with w [64][256] (K order
// tap-major, channel-minor), 16-bit; stats (nullable) [Nb*H][3][64] shifted partials per output
// row (W rows of M). Requires H % 4 == 0, W % 16 == 0, W <= 128; returns -1 otherwise.
extern "C" int pda_stem_fwd(const void* x, const void* w, void* y, float* stats, int Nb, int H, int W,
                            int dt, int grid_cap, hipStream_t st) {
  if (Nb <= 0 || H <= 0 || H % ST_TH || W % 16 || W < 16 || W > 128 || (dt != DT_BF16 && dt != DT_F16))
    return -1;
#define STEM_CASE(PFV)                                                                              \
  case PFV:                                                                                         \
    return dt == DT_BF16 ? launch_stem<DT_BF16, PFV>(x, w, y, stats, Nb, H, grid_cap, st)           \
                         : launch_stem<DT_F16, PFV>(x, w, y, stats, Nb, H, grid_cap, st);
  switch (W / 16) {
    STEM_CASE(1) STEM_CASE(2) STEM_CASE(3) STEM_CASE(4)
    STEM_CASE(5) STEM_CASE(6) STEM_CASE(7) STEM_CASE(8)
  }
#undef STEM_CASE
  return -1;
}
