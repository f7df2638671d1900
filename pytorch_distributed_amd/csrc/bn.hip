// BatchNorm (+ReLU, +residual, +pool) kernels for gfx950, NHWC bf16/f16 (or exact-f32) activations,
// f32 statistics.
//
// Replaces cuDNN BatchNorm train fwd/bwd + ATen ReLU/threshold_backward/add/max_pool2d/avg_pool2d
// of the reference stack. Statistics are computed from the conv
// epilogue's per-tile partial sums (conv_gemm.hip) or by the column-reduce kernel below; every
// cross-workgroup sum is a deterministic slab reduction (no float atomics).
//
//   bn_finalize_tot : f64 totals [2][C] -> mean, invstd, scale = g*invstd, shift = b - mean*scale,
//                     running-stat update (momentum, unbiased var), num_batches_tracked += 1
//   bn_apply        : a = act(y*scale + shift [+ res | + y2*scale2 + shift2]), 16 B / lane
//   stem_pool       : a = relu(bn(y)) then 3x3/s2/p1 max-pool with a uint8 argmax per output
//   tail_pool       : a = relu(bn3(y3) + shortcut) then global average pool (head of ResNet)
//   bn_bwd_reduce   : partials of sum(dz), sum(dz*xhat) [, sum(dz*xhat_ds)] with dz = dA*mask
//   bn_bwd_finalize : gamma/beta grads into the flat gradient buffer + apply coefficients
//   bn_bwd_apply    : dy = k1*dz + k2*y + k3 (dz recomputed, or read back from the tail buffer)
//   maxpool_bwd     : deterministic gather of max-pool gradients through the argmax bytes
#include "common.h"

#include <cstdlib>
#include <cstring>

namespace {

constexpr int NT = 256;

__device__ __forceinline__ void ld8f(const float* p, float* f) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  f[0] = a[0]; f[1] = a[1]; f[2] = a[2]; f[3] = a[3];
  f[4] = b[0]; f[5] = b[1]; f[6] = b[2]; f[7] = b[3];
}

// ------------------------------------------------------------------ finalize helpers
// Sum of slabs t = g, g+64, ... of two per-channel columns (o0, o1) of a [T][pitch] partial buffer
// in f64, with four independent load chains (the loads pipeline instead of serialising on one
// accumulator). The summation order depends only on T: deterministic.
__device__ __forceinline__ void slab_sum2(const float* __restrict__ part, int T, int pitch, int o0,
                                          int o1, int g, double& s0, double& s1) {
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0, b0 = 0.0, b1 = 0.0, b2 = 0.0, b3 = 0.0;
  int t = g;
  for (; t + 192 < T; t += 256) {
    a0 += part[(size_t)t * pitch + o0];         b0 += part[(size_t)t * pitch + o1];
    a1 += part[(size_t)(t + 64) * pitch + o0];  b1 += part[(size_t)(t + 64) * pitch + o1];
    a2 += part[(size_t)(t + 128) * pitch + o0]; b2 += part[(size_t)(t + 128) * pitch + o1];
    a3 += part[(size_t)(t + 192) * pitch + o0]; b3 += part[(size_t)(t + 192) * pitch + o1];
  }
  for (; t < T; t += 64) {
    a0 += part[(size_t)t * pitch + o0];
    b0 += part[(size_t)t * pitch + o1];
  }
  s0 = (a0 + a1) + (a2 + a3);
  s1 = (b0 + b1) + (b2 + b3);
}

// fixed-shape tree over the 64 partial-lanes of red[2][64][17] (1024-thread block: g = tid >> 4,
// cl = tid & 15); red[q][0][cl] holds the totals afterwards. Replaces a 64-step serial LDS walk.
__device__ __forceinline__ void tree_reduce2(double (&red)[2][64][17], int g, int cl) {
  __syncthreads();
#pragma unroll
  for (int s = 32; s > 0; s >>= 1) {
    if (g < s) {
      red[0][g][cl] += red[0][g + s][cl];
      red[1][g][cl] += red[1][g + s][cl];
    }
    __syncthreads();
  }
}

// ------------------------------------------------------------------ forward finalize
// From f64 totals tot[2][C] = (sum y, sum y^2) of the conv forward (bn_fwd_stats with a totals
// buffer), after the SyncBatchNorm all-reduce.
__global__ __launch_bounds__(256) void bn_finalize_tot_kernel(
    const double* __restrict__ tot, int C, double count, const float* __restrict__ gamma,
    const float* __restrict__ beta, float eps, float momentum, float* __restrict__ mean_out,
    float* __restrict__ invstd_out, float* __restrict__ scale, float* __restrict__ shift,
    float* __restrict__ run_mean, float* __restrict__ run_var, long long* __restrict__ nbt,
    int update_running) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c < C) {
    const double mean = tot[c] / count;
    double var = tot[C + c] / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float inv = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * inv;
    mean_out[c] = (float)mean;
    invstd_out[c] = inv;
    scale[c] = sc;
    shift[c] = beta[c] - (float)mean * sc;
    if (update_running) {
      const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
      run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
      run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unb;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && update_running && nbt) *nbt += 1;
}

// BatchNorm statistics from per-tile partial sums, finalized in ONE launch (no separate
// reduce / finalize launches, no float atomics, deterministic):
//   KIND 0 (forward): the conv epilogue's SHIFTED partials part[T][3][C] = (sum(y-s), sum((y-s)^2),
//          s) over tiles of `bm` rows (the last one ragged) -> mean / invstd / scale / shift /
//          running statistics (or, SyncBatchNorm, f64 totals for the all-reduce);
//   KIND 1 (backward): the dgrad epilogue's partials part[T][NQ][C] = (sum dz, sum dz*y
//          [, sum dz*y2]) -> gamma / beta gradients + apply coefficients k of each BN branch.
// Block (s, g) reduces tiles [s*T/S, (s+1)*T/S) of channel group g (CG = min(C, 256) channels) to
// an f64 slab -- 16-B loads, (channel quad x slab lane) threads, fixed-order lane combine -- and
// publishes it write-through (sc1 stores, vmcnt(0), barrier, agent-scope arrival counter); the
// group's last arriving block (agent acquire) sums the S slabs in slab order and finalizes.
struct BnFwdOut {  // mirrors ops/ext.py BnFwdOut
  const float* gamma; const float* beta;
  float eps, momentum;
  float* mean; float* invstd; float* scale; float* shift;
  float* rmean; float* rvar; long long* nbt;
  int update;
  double* tot;   // non-null: f64 totals [2][C] instead of the finalize (bn_finalize_tot after)
};

struct BnBwdOut {  // mirrors ops/ext.py BnBwdOut; branch b = 0: BN of y, 1: shortcut BN of y2
  float count, gscale;
  int accumulate;
  const float* gamma[2]; const float* mean[2]; const float* invstd[2];
  float* dgamma[2]; float* dbeta[2];
  float* k;      // [NQ-1][3][C]: dy_b = k0*dz + k1*y_b + k2
};

__device__ __forceinline__ void st_wt(double* q, double v) {   // write-through (sc1) store
  __hip_atomic_store(q, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// tiles / slabs whose loads each lane keeps in flight together (levels 1 / 2)
#ifndef BN_STATS_U1
#define BN_STATS_U1 4
#endif
#ifndef BN_STATS_U2
#define BN_STATS_U2 4
#endif
template <int KIND, int NQ, class Out>
__global__ __launch_bounds__(256) void bn_stats_kernel(const float* __restrict__ part, int T, int C,
                                                       int bm, int M, int CG,
                                                       double* __restrict__ slabs,
                                                       int* __restrict__ cnt, Out o) {
  // 8 KiB of LDS whatever NQ: the kernel runs on the main stream beside the weight-gradient
  // GEMMs, whose LDS-DMA tiles hold 144 KiB of a CU's 160 KiB -- a larger footprint could only be
  // placed on CUs with no weight-gradient block resident (measured: 150-180 us instead of ~15 us)
  __shared__ double red[1024];   // [(lane * Q + quad) * 4 + e] of one q at a time
  __shared__ int flag;
  const int S = gridDim.x, s = blockIdx.x, g = blockIdx.y, tid = threadIdx.x;
  const int Q = CG >> 2, SL = 256 / Q;
  const int quad = tid % Q, lane = tid / Q;
  const int c = g * CG + quad * 4;
  const bool act = lane < SL && c < C;
  // fixed-order sum over the SL lanes of each column v < CG of this group: thread v gets tot[q]
  double tot[NQ];
  auto combine = [&](const double (&a)[NQ][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      __syncthreads();
#pragma unroll
      for (int e = 0; e < 4; ++e) red[tid * 4 + e] = a[q][e];
      __syncthreads();
      double sum = 0.0;
      if (tid < CG) {
        const int qi = tid >> 2, e = tid & 3;
        for (int l = 0; l < SL; ++l) sum += red[(l * Q + qi) * 4 + e];
      }
      tot[q] = sum;
    }
  };
  constexpr int PQ = KIND == 0 ? 3 : NQ;   // partial rows per tile
  {  // level 1: this block's tiles -> slab s
    double a[NQ][4];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[q][e] = 0.0;
    const int t0 = (int)((long long)s * T / S), t1 = (int)((long long)(s + 1) * T / S);
    if (act) {
      // U1 tiles' loads issued before the first use (the compiler kept one iteration's loads in
      // flight per lane -- a dependent round per tile, ~1.5 us each beside the weight-gradient
      // stream); accumulated in the same t order as before: bit-identical sums
      auto acc1 = [&](const f32x4 (&d)[PQ], int tu) __attribute__((always_inline)) {
        if constexpr (KIND == 0) {
          const double rows = (double)min(bm, M - tu * bm);
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const double s_ = d[2][e], x = d[0][e];
            a[0][e] += rows * s_ + x;
            a[1][e] += (double)d[1][e] + s_ * (2.0 * x + rows * s_);
          }
        } else {
#pragma unroll
          for (int q = 0; q < NQ; ++q)
#pragma unroll
            for (int e = 0; e < 4; ++e) a[q][e] += (double)d[q][e];
        }
      };
      int t = t0 + lane;
      for (; t + (BN_STATS_U1 - 1) * SL < t1; t += SL * BN_STATS_U1) {   // whole batches
        f32x4 d[BN_STATS_U1][PQ];
#pragma unroll
        for (int u = 0; u < BN_STATS_U1; ++u) {
          const float* pt = part + (size_t)(t + u * SL) * PQ * C + c;
#pragma unroll
          for (int q = 0; q < PQ; ++q) d[u][q] = *reinterpret_cast<const f32x4*>(pt + q * C);
        }
#pragma unroll
        for (int u = 0; u < BN_STATS_U1; ++u) acc1(d[u], t + u * SL);
      }
      for (; t < t1; t += SL) {   // the rest, one tile at a time
        f32x4 d[PQ];
        const float* pt = part + (size_t)t * PQ * C + c;
#pragma unroll
        for (int q = 0; q < PQ; ++q) d[q] = *reinterpret_cast<const f32x4*>(pt + q * C);
        acc1(d, t);
      }
    }
    combine(a);
    const int col = g * CG + tid;
    if (tid < CG && col < C)
#pragma unroll
      for (int q = 0; q < NQ; ++q) st_wt(slabs + ((size_t)s * NQ + q) * C + col, tot[q]);
  }
  // arrival: the slab was stored write-through (sc1, st_wt) and every wave drains its stores
  // (vmcnt(0)) before the barrier, then ONE relaxed agent-scope arrival on the group counter --
  // the sc1 form of the hand-off (cdna_hip_programming.md G16 / the in-launch split-K recipe): no
  // release fence, whose buffer_wbl2 writes back the XCD L2's dirty lines -- in the step, the
  // streaming kernels' output beside this launch (BN_STATS_RELEASE=1 restores it)
#ifndef BN_STATS_RELEASE
#define BN_STATS_RELEASE 0
#endif
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    if constexpr (BN_STATS_RELEASE) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    const int old = __hip_atomic_fetch_add(cnt + g, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    flag = old == S - 1;
  }
  __syncthreads();
  if (!flag) return;
  if (tid == 0) {
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __hip_atomic_store(cnt + g, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);   // reset
  }
  __syncthreads();
  {  // level 2 (the group's last arriver): the S slabs, in slab order per lane
    double a[NQ][4];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 4; ++e) a[q][e] = 0.0;
    constexpr int U2 = NQ > 2 ? BN_STATS_U2 / 2 : BN_STATS_U2;
    if (act)
      {
        auto acc2 = [&](const f64x2 (&x)[NQ][2]) __attribute__((always_inline)) {
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            a[q][0] += x[q][0][0]; a[q][1] += x[q][0][1];
            a[q][2] += x[q][1][0]; a[q][3] += x[q][1][1];
          }
        };
        auto ld2 = [&](f64x2 (&x)[NQ][2], int tu) __attribute__((always_inline)) {
#pragma unroll
          for (int q = 0; q < NQ; ++q) {
            const double* p0 = slabs + ((size_t)tu * NQ + q) * C + c;
            x[q][0] = *reinterpret_cast<const f64x2*>(p0);
            x[q][1] = *reinterpret_cast<const f64x2*>(p0 + 2);
          }
        };
        int t = lane;
        for (; t + (U2 - 1) * SL < S; t += SL * U2) {   // whole batches of U2 slabs
          f64x2 x[U2][NQ][2];
#pragma unroll
          for (int u = 0; u < U2; ++u) ld2(x[u], t + u * SL);
#pragma unroll
          for (int u = 0; u < U2; ++u) acc2(x[u]);
        }
        for (; t < S; t += SL) {
          f64x2 x[NQ][2];
          ld2(x, t);
          acc2(x);
        }
      }
    combine(a);
  }
  const int col = g * CG + tid;
  if (tid < CG && col < C) {
    if constexpr (KIND == 0) {
      const double sx = tot[0], sxx = tot[1];
      if (o.tot) {
        o.tot[col] = sx;
        o.tot[C + col] = sxx;
      } else {
        const double count = (double)M;
        const double mean = sx / count;
        double var = sxx / count - mean * mean;
        if (var < 0.0) var = 0.0;
        const float inv = (float)(1.0 / sqrt(var + (double)o.eps));
        const float sc = o.gamma[col] * inv;
        o.mean[col] = (float)mean;
        o.invstd[col] = inv;
        o.scale[col] = sc;
        o.shift[col] = o.beta[col] - (float)mean * sc;
        if (o.update) {
          const double unb = count > 1.0 ? var * count / (count - 1.0) : var;
          o.rmean[col] = (1.f - o.momentum) * o.rmean[col] + o.momentum * (float)mean;
          o.rvar[col] = (1.f - o.momentum) * o.rvar[col] + o.momentum * (float)unb;
        }
      }
    } else {
      const double count = o.count, gs = o.gscale, sdz = tot[0];
#pragma unroll
      for (int b = 0; b < NQ - 1; ++b) {   // constant member indices (no dynamic param indexing)
        const double mu = o.mean[b][col], is = o.invstd[b][col], ga = o.gamma[b][col];
        const double sdzx = (tot[1 + b] - mu * sdz) * is;   // sum dz * xhat
        float* dg = o.dgamma[b];
        float* db = o.dbeta[b];
        dg[col] = (float)(sdzx * gs) + (o.accumulate ? dg[col] : 0.f);
        db[col] = (float)(sdz * gs) + (o.accumulate ? db[col] : 0.f);
        const double ak = ga * is;
        const double kk2 = -ak * is * sdzx / count;
        float* k = o.k + (size_t)b * 3 * C;
        k[col] = (float)ak;
        k[C + col] = (float)kk2;
        k[2 * C + col] = (float)(-ak * sdz / count - kk2 * mu);
      }
    }
  }
  if constexpr (KIND == 0)
    if (g == 0 && tid == 0 && !o.tot && o.update && o.nbt) *o.nbt += 1;
}

// eval-mode scale/shift from running statistics
__global__ void bn_eval_coeffs_kernel(const float* __restrict__ gamma, const float* __restrict__ beta,
                                      const float* __restrict__ rm, const float* __restrict__ rv,
                                      float eps, int C, float* __restrict__ scale,
                                      float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float inv = rsqrtf(rv[c] + eps);
  scale[c] = gamma[c] * inv;
  shift[c] = beta[c] - rm[c] * gamma[c] * inv;
}

// ------------------------------------------------------------------ apply
// mode: 0 = act(bn(y)); 1 = act(bn(y) + res); 2 = act(bn(y) + bn2(y2))
template <int DT>
__device__ __forceinline__ void ld8p(const float* p, f32x2* f) {
  const f32x4 a = *reinterpret_cast<const f32x4*>(p);
  const f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
  f[0] = f32x2{a[0], a[1]}; f[1] = f32x2{a[2], a[3]};
  f[2] = f32x2{b[0], b[1]}; f[3] = f32x2{b[2], b[3]};
}

// Streaming form: 32-bit indices; when the grid stride is a multiple of C/8 (always for
// power-of-two C <= 2048 with 256-thread blocks) each thread's channel chunk is loop-invariant,
// so the per-channel coefficients are loaded once, and the math runs on packed pairs.
template <int DT>
__global__ __launch_bounds__(NT) void bn_apply_kernel(
    const void* __restrict__ y, const float* __restrict__ sc, const float* __restrict__ sh,
    const void* __restrict__ r2, const float* __restrict__ sc2, const float* __restrict__ sh2,
    void* __restrict__ out, int n8, int C, int mode, int relu, uint8_t* __restrict__ mask) {
  const int C8 = C >> 3;
  const int stride = gridDim.x * NT;
  const bool fixed = (stride % C8) == 0;
  int i = blockIdx.x * NT + threadIdx.x;
  f32x2 a[4], b[4], a2[4], b2[4];
  int cprev = -1;
  for (; i < n8; i += stride) {
    const int c0 = (i % C8) * 8;
    if (!fixed || cprev < 0) {
      ld8p<DT>(sc + c0, a);
      ld8p<DT>(sh + c0, b);
      if (mode == 2) {
        ld8p<DT>(sc2 + c0, a2);
        ld8p<DT>(sh2 + c0, b2);
      }
      cprev = c0;
    }
    if constexpr (DT == DT_F32) {
      float yv[8], rv[8], o[8];
      load8<DT>(y, (size_t)i * 8, yv);
      if (mode) load8<DT>(r2, (size_t)i * 8, rv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float v = yv[e] * a[e >> 1][e & 1] + b[e >> 1][e & 1];
        if (mode) v += mode == 2 ? rv[e] * a2[e >> 1][e & 1] + b2[e >> 1][e & 1] : rv[e];
        o[e] = relu ? fmaxf(v, 0.f) : v;
      }
      store8<DT>(out, (size_t)i * 8, o);
      if (mask) {
        uint32_t bits = 0;
#pragma unroll
        for (int e = 0; e < 8; ++e) bits |= (o[e] > 0.f ? 1u : 0u) << e;
        mask[i] = (uint8_t)bits;
      }
      continue;
    }
    const i32x4 yv = reinterpret_cast<const i32x4*>(y)[i];
    i32x4 rv = {0, 0, 0, 0};
    if (mode) rv = reinterpret_cast<const i32x4*>(r2)[i];
    i32x4 o;
    uint32_t bits = 0;   // ReLU mask of the output (bit e = element e > 0), for the backward
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x2 v = tail_pre2(unpack2<DT>((uint32_t)yv[k]), a[k], b[k], unpack2<DT>((uint32_t)rv[k]),
                          a2[k], b2[k], mode);
      if (relu) v = f32x2{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f)};
      o[k] = (int)pack2<DT>(v);
      bits |= (v.x > 0.f ? 1u : 0u) << (2 * k);
      bits |= (v.y > 0.f ? 1u : 0u) << (2 * k + 1);
    }
    reinterpret_cast<i32x4*>(out)[i] = o;
    if (mask) mask[i] = (uint8_t)bits;
  }
}

// ------------------------------------------------------------------ stem: bn + relu + maxpool 3x3/2/1
// y: [N,H,W,C], out: [N,Ho,Wo,C], arg: [N,Ho,Wo,C] uint8 window index (0..8)
template <int DT>
__global__ __launch_bounds__(NT) void stem_pool_kernel(const void* __restrict__ y,
                                                       const float* __restrict__ sc,
                                                       const float* __restrict__ sh,
                                                       void* __restrict__ out,
                                                       uint8_t* __restrict__ arg, int N, int H,
                                                       int W, int C, int Ho, int Wo, FastDiv dCK,
                                                       FastDiv dWo, FastDiv dHo, int rev) {
  const int CK = C / 8;
  const int total = N * Ho * Wo * CK;
  for (int i0 = blockIdx.x * NT + threadIdx.x; i0 < total; i0 += gridDim.x * NT) {
    // rev: last rows first -- the stem conv wrote them last, so up to the Infinity Cache's 256 MiB
    // of y are still cached when the pool starts
    const int i = rev ? total - 1 - i0 : i0;
    const uint32_t pix = fdiv(i, dCK), ck = i - pix * CK;
    const uint32_t p2 = fdiv(pix, dWo), xo = pix - p2 * Wo;
    const uint32_t n = fdiv(p2, dHo), yo = p2 - n * Ho;
    float a[8], b[8], best[8];
    int bi[8];
    ld8f(sc + ck * 8, a);
    ld8f(sh + ck * 8, b);
#pragma unroll
    for (int e = 0; e < 8; ++e) { best[e] = -1.f; bi[e] = 0; }
    for (int dy = 0; dy < 3; ++dy) {
      const int yy = yo * 2 - 1 + dy;
      if ((unsigned)yy >= (unsigned)H) continue;
      for (int dx = 0; dx < 3; ++dx) {
        const int xx = xo * 2 - 1 + dx;
        if ((unsigned)xx >= (unsigned)W) continue;
        float v[8];
        load8<DT>(y, ((n * H + yy) * W + xx) * C + ck * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float r = fmaxf(v[e] * a[e] + b[e], 0.f);
          if (r > best[e]) { best[e] = r; bi[e] = dy * 3 + dx; }
        }
      }
    }
    store8<DT>(out, (size_t)i * 8, best);
    uint64_t packed = 0;
#pragma unroll
    for (int e = 0; e < 8; ++e) packed |= (uint64_t)bi[e] << (8 * e);
    reinterpret_cast<uint64_t*>(arg)[i] = packed;
  }
}

// gradient of relu(bn(y)) through the max-pool: dA[n,y,x,c] = sum over windows whose argmax is here
template <int DT>
__global__ __launch_bounds__(NT) void maxpool_bwd_kernel(const void* __restrict__ dout,
                                                         const void* __restrict__ dout2,
                                                         const uint8_t* __restrict__ arg,
                                                         void* __restrict__ din, int N, int H, int W,
                                                         int C, int Ho, int Wo, FastDiv dCK,
                                                         FastDiv dW, FastDiv dH) {
  const int CK = C / 8;
  const int total = N * H * W * CK;
  for (int i = blockIdx.x * NT + threadIdx.x; i < total; i += gridDim.x * NT) {
    const uint32_t pix = fdiv(i, dCK), ck = i - pix * CK;
    const uint32_t p2 = fdiv(pix, dW), x = pix - p2 * W;
    const uint32_t n = fdiv(p2, dH), yy = p2 - n * H;
    float g[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] = 0.f;
    // outputs whose window covers (yy, x): yo*2-1 <= yy <= yo*2+1
    for (int yo = (int)yy / 2; yo <= min(Ho - 1, ((int)yy + 1) / 2); ++yo) {
      const int dy = (int)yy - (yo * 2 - 1);
      if (dy < 0 || dy > 2) continue;
      for (int xo = (int)x / 2; xo <= min(Wo - 1, ((int)x + 1) / 2); ++xo) {
        const int dx = (int)x - (xo * 2 - 1);
        if (dx < 0 || dx > 2) continue;
        const uint32_t o = (n * Ho + yo) * Wo + xo;
        const uint64_t a = reinterpret_cast<const uint64_t*>(arg)[o * CK + ck];
        float d[8];
        load8<DT>(dout, o * C + ck * 8, d);
        if (dout2) {
          float d2[8];
          load8<DT>(dout2, o * C + ck * 8, d2);
#pragma unroll
          for (int e = 0; e < 8; ++e) d[e] += d2[e];
        }
        const int me = dy * 3 + dx;
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if ((int)((a >> (8 * e)) & 0xff) == me) g[e] += d[e];
      }
    }
    store8<DT>(din, (size_t)i * 8, g);
  }
}

// ------------------------------------------------------------------ head: tail + global avg pool
// out[n][c] = mean_{hw} relu(bn3(y3) + shortcut) ; shortcut: mode 1 = res tensor, 2 = bn_ds(y_ds)
template <int DT>
__global__ __launch_bounds__(NT) void tail_pool_kernel(const void* __restrict__ y,
                                                       const float* __restrict__ sc,
                                                       const float* __restrict__ sh,
                                                       const void* __restrict__ r2,
                                                       const float* __restrict__ sc2,
                                                       const float* __restrict__ sh2,
                                                       void* __restrict__ out, int HW, int C,
                                                       int mode) {
  const int n = blockIdx.x;
  const int CK = C / 8;
  for (int ck = threadIdx.x; ck < CK; ck += NT) {
    float a[8], b[8], a2[8], b2[8], acc[8];
    ld8f(sc + ck * 8, a);
    ld8f(sh + ck * 8, b);
    if (mode == 2) {
      ld8f(sc2 + ck * 8, a2);
      ld8f(sh2 + ck * 8, b2);
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    for (int pp = 0; pp < HW; ++pp) {
      const size_t off = ((size_t)n * HW + pp) * C + ck * 8;
      float v[8], w[8];
      load8<DT>(y, off, v);
      load8<DT>(r2, off, w);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float s = w[e];
        if (mode == 2) s = s * a2[e] + b2[e];
        acc[e] += fmaxf(v[e] * a[e] + b[e] + s, 0.f);
      }
    }
    const float inv = 1.f / (float)HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] *= inv;
    store8<DT>(out, (size_t)n * C + ck * 8, acc);
  }
}

// ------------------------------------------------------------------ backward reduce
// dA = g1 (+ g2), or, when pooled (HW > 0), dA[n,p,c] = gp[n][c] / HW.
// mask mode: 0 = relu on bn(y) (bn1/bn2/stem), 1 = relu on bn(y)+res, 2 = relu on bn(y)+bn2(y2),
//            3 = no mask (dz given in g1, e.g. downsample branch re-reading the tail's dz)
// Outputs partials [G][NQ][C]: q0 = sum dz, q1 = sum dz*y, q2 = sum dz*y2 (mode 2); dz stored if dz_out.
struct BwdArgs {
  const void* g1; const void* g2; const void* gp; int HW;
  const void* y; const float* sc; const float* sh;
  const void* y2; const float* sc2; const float* sh2;
  int mode;
  void* dz_out;
  float* part; int nq;
  long long rows; int C;
  long long rows_per_block;
};

template <int DT>
__device__ __forceinline__ void load_grad(const BwdArgs& a, long long row, int c0, float* g) {
  if (a.gp) {
    const long long n = row / a.HW;
    load8<DT>(a.gp, n * a.C + c0, g);
    const float inv = 1.f / (float)a.HW;
#pragma unroll
    for (int e = 0; e < 8; ++e) g[e] *= inv;
  } else {
    load8<DT>(a.g1, row * a.C + c0, g);
    if (a.g2) {
      float h[8];
      load8<DT>(a.g2, row * a.C + c0, h);
#pragma unroll
      for (int e = 0; e < 8; ++e) g[e] += h[e];
    }
  }
}

// dz for one 8-channel chunk of row; also returns y (and y2) values for the moment sums
template <int DT>
__device__ __forceinline__ void make_dz(const BwdArgs& a, long long row, int c0, float* dz,
                                        float* yv, float* y2v) {
  load_grad<DT>(a, row, c0, dz);
  load8<DT>(a.y, row * a.C + c0, yv);
  if (a.mode == 3) return;
  float s[8], h[8];
  ld8f(a.sc + c0, s);
  ld8f(a.sh + c0, h);
  float pre[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) pre[e] = yv[e] * s[e] + h[e];
  if (a.mode >= 1) {
    load8<DT>(a.y2, row * a.C + c0, y2v);
    if (a.mode == 2) {
      ld8f(a.sc2 + c0, s);
      ld8f(a.sh2 + c0, h);
#pragma unroll
      for (int e = 0; e < 8; ++e) pre[e] += y2v[e] * s[e] + h[e];
    } else {
#pragma unroll
      for (int e = 0; e < 8; ++e) pre[e] += y2v[e];
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) dz[e] = pre[e] > 0.f ? dz[e] : 0.f;
}

template <int DT>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_kernel(BwdArgs a) {
  __shared__ float red[3][NT][8];
  const int CK = a.C / 8;
  const int tpr = CK < NT ? CK : NT;       // threads per row
  const int rpi = NT / tpr;                // rows per iteration
  const int ck = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  const long long r0 = blockIdx.x * a.rows_per_block;
  const long long r1 = min(a.rows, r0 + a.rows_per_block);
  for (int cbase = 0; cbase < CK; cbase += tpr) {
    const int c0 = (cbase + ck) * 8;
    float q0[8], q1[8], q2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { q0[e] = 0.f; q1[e] = 0.f; q2[e] = 0.f; }
    if (threadIdx.x < tpr * rpi) {
      for (long long row = r0 + rsub; row < r1; row += rpi) {
        float dz[8], yv[8], y2v[8];
        make_dz<DT>(a, row, c0, dz, yv, y2v);
        if (a.dz_out) store8<DT>(a.dz_out, row * a.C + c0, dz);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          q0[e] += dz[e];
          q1[e] += dz[e] * yv[e];
        }
        if (a.nq > 2) {
#pragma unroll
          for (int e = 0; e < 8; ++e) q2[e] += dz[e] * y2v[e];
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][threadIdx.x][e] = q0[e];
      red[1][threadIdx.x][e] = q1[e];
      red[2][threadIdx.x][e] = q2[e];
    }
    __syncthreads();
    if (threadIdx.x < tpr) {
      for (int q = 0; q < a.nq; ++q) {
        float s[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) s[e] = 0.f;
        for (int r = 0; r < rpi; ++r)
#pragma unroll
          for (int e = 0; e < 8; ++e) s[e] += red[q][r * tpr + threadIdx.x][e];
        float* dst = a.part + ((size_t)blockIdx.x * a.nq + q) * a.C + c0;
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = s[e];
      }
    }
    __syncthreads();
  }
}

// Stem backward, one pass: maxpool gradient gather (as maxpool_bwd_kernel) -> ReLU mask of
// relu(bn(y0)) -> dz stored -> per-block partials q0 = sum dz, q1 = sum dz*y0. Replaces
// maxpool_bwd (write dA0) + bn_bwd_reduce (re-read dA0): one full read of the largest activation
// of the network (400x112x112x64) less, and one launch less.
// Work item = one 2x2 quad of input pixels (2yo..2yo+1, 2xo..2xo+1) x 8 channels: the pooling
// windows covering it are exactly (yo..yo+1) x (xo..xo+1) (3x3/2, pad 1), so each window's argmax
// bytes and gradient(s) are gathered ONCE per quad instead of once per pixel (4x less gather
// traffic; the per-pixel form was request-bound at ~190 B of loads per 16 B stored).
template <int DT>
__global__ __launch_bounds__(NT) void stem_bwd_reduce_kernel(
    const void* __restrict__ dout, const void* __restrict__ dout2, const uint8_t* __restrict__ arg,
    const void* __restrict__ y, const float* __restrict__ sc, const float* __restrict__ sh,
    void* __restrict__ dz_out, float* __restrict__ part, long long quads, long long quads_per_block,
    int H, int W, int C, int Ho, int Wo, FastDiv dWo, FastDiv dHo) {
  __shared__ float red[2][NT][8];
  const int CK = C / 8;
  const int tpr = CK < NT ? CK : NT;
  const int rpi = NT / tpr;
  const int ck = threadIdx.x % tpr, rsub = threadIdx.x / tpr;
  const long long r0 = blockIdx.x * quads_per_block;
  const long long r1 = min(quads, r0 + quads_per_block);
  for (int cbase = 0; cbase < CK; cbase += tpr) {
    const int cc = cbase + ck, c0 = cc * 8;
    float q0[8], q1[8], s[8], h[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) { q0[e] = 0.f; q1[e] = 0.f; }
    ld8f(sc + c0, s);
    ld8f(sh + c0, h);
    if (threadIdx.x < tpr * rpi) {
      // two quads in flight per thread: 520-529 vs 540-554 us in the step (x4: 572-593 us,
      // tools/gpu_kernel_ab.sh; profiles/ab_r3_dma.md section 20)
#pragma unroll 2
      for (long long qd = r0 + rsub; qd < r1; qd += rpi) {
        const uint32_t p2 = fdiv((uint32_t)qd, dWo), xo = (uint32_t)qd - p2 * Wo;
        const uint32_t n = fdiv(p2, dHo), yo = p2 - n * Ho;
        const bool y1 = (int)yo + 1 < Ho, x1 = (int)xo + 1 < Wo;
        // gather the 4 windows (w bit 1: yo+1, bit 0: xo+1); a window past the edge re-reads a
        // valid one and gets argmax bytes 0xff, which match no tap
        Raw8<DT> dv[4], dv2[4];
        uint64_t am[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          const bool live = ((w & 2) == 0 || y1) && ((w & 1) == 0 || x1);
          const uint32_t o = (n * Ho + yo + ((w & 2) && y1 ? 1 : 0)) * Wo + xo + ((w & 1) && x1 ? 1 : 0);
          const uint64_t a8 = reinterpret_cast<const uint64_t*>(arg)[o * CK + cc];
          am[w] = live ? a8 : ~0ull;
          dv[w] = ldraw8<DT>(dout, (size_t)o * C + c0);
          if (dout2) dv2[w] = ldraw8<DT>(dout2, (size_t)o * C + c0);
        }
        // the quad's 4 pixels (pixel bit 1: row 2yo+1, bit 0: col 2xo+1); a pixel past an odd
        // edge loads the quad's first pixel and is neither stored nor counted
        Raw8<DT> yr[4];
        bool pin[4];
        size_t prow[4];
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          const int yy = 2 * (int)yo + (px >> 1), x = 2 * (int)xo + (px & 1);
          pin[px] = yy < H && x < W;
          prow[px] = ((size_t)n * H + (pin[px] ? yy : 2 * (int)yo)) * W + (pin[px] ? x : 2 * (int)xo);
          yr[px] = ldraw8<DT>(y, prow[px] * C + c0);
        }
        float d[4][8];
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          cvt8<DT>(dv[w], d[w]);
          if (dout2) {
            float d2[8];
            cvt8<DT>(dv2[w], d2);
#pragma unroll
            for (int e = 0; e < 8; ++e) d[w][e] += d2[e];
          }
        }
#pragma unroll
        for (int px = 0; px < 4; ++px) {
          const int py = px >> 1, pxx = px & 1;
          float g[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = 0.f;
#pragma unroll
          for (int w = 0; w < 4; ++w) {
            const int wy = w >> 1, wx = w & 1;
            // window (yo+wy) covers rows 2(yo+wy)-1 .. 2(yo+wy)+1: pixel row 2yo+py is inside iff
            // py - 2wy >= -1, i.e. not (py = 0, wy = 1); same for columns (compile-time)
            if ((wy && !py) || (wx && !pxx)) continue;
            const int me = (py + 1 - 2 * wy) * 3 + (pxx + 1 - 2 * wx);
#pragma unroll
            for (int e = 0; e < 8; ++e)
              if ((int)((am[w] >> (8 * e)) & 0xff) == me) g[e] += d[w][e];
          }
          float yv[8];
          cvt8<DT>(yr[px], yv);
#pragma unroll
          for (int e = 0; e < 8; ++e) g[e] = yv[e] * s[e] + h[e] > 0.f ? g[e] : 0.f;
          if (!pin[px]) continue;
          // statistics of the stored (rounded) dz, as the apply kernel re-reads it
          const Raw8<DT> pk = pk8<DT>(g);
          straw8<DT>(dz_out, prow[px] * C + c0, pk);
          cvt8<DT>(pk, g);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            q0[e] += g[e];
            q1[e] += g[e] * yv[e];
          }
        }
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red[0][threadIdx.x][e] = q0[e];
      red[1][threadIdx.x][e] = q1[e];
    }
    __syncthreads();
    if (threadIdx.x < tpr) {
      for (int q = 0; q < 2; ++q) {
        float t[8];
#pragma unroll
        for (int e = 0; e < 8; ++e) t[e] = 0.f;
        for (int r = 0; r < rpi; ++r)
#pragma unroll
          for (int e = 0; e < 8; ++e) t[e] += red[q][r * tpr + threadIdx.x][e];
        float* dst = part + ((size_t)blockIdx.x * 2 + q) * C + c0;
#pragma unroll
        for (int e = 0; e < 8; ++e) dst[e] = t[e];
      }
    }
    __syncthreads();
  }
}

// finalize: for branch b (0: y with q0,q1; 1: y2 with q0,q2) produce gamma/beta grads and
// coefficients k1,k2,k3 such that dy = k1*dz + k2*y + k3.
__global__ __launch_bounds__(1024) void bn_bwd_finalize_kernel(
    const float* __restrict__ part, int G, int nq, int qy, int C, float count,
    const float* __restrict__ gamma, const float* __restrict__ mean, const float* __restrict__ invstd,
    float* __restrict__ dgamma, float* __restrict__ dbeta, float* __restrict__ k1,
    float* __restrict__ k2, float* __restrict__ k3, float gscale, int accumulate) {
  __shared__ double red[2][64][17];
  const int cl = threadIdx.x & 15, g = threadIdx.x >> 4;
  const int c = blockIdx.x * 16 + cl;
  double s0 = 0.0, s1 = 0.0;
  if (c < C) slab_sum2(part, G, nq * C, c, qy * C + c, g, s0, s1);
  red[0][g][cl] = s0;
  red[1][g][cl] = s1;
  tree_reduce2(red, g, cl);
  if (g == 0 && c < C) {
    const double sdz = red[0][0][cl], sdzy = red[1][0][cl];
    const double mu = mean[c], is = invstd[c], ga = gamma[c];
    const double sdzx = (sdzy - mu * sdz) * is;  // sum dz * xhat
    dgamma[c] = (float)(sdzx * gscale) + (accumulate ? dgamma[c] : 0.f);
    dbeta[c] = (float)(sdz * gscale) + (accumulate ? dbeta[c] : 0.f);
    const double a = ga * is;
    const double kk2 = -a * is * sdzx / count;
    k1[c] = (float)a;
    k2[c] = (float)kk2;
    k3[c] = (float)(-a * sdz / count - kk2 * mu);
  }
}

// dy = k1*dz + k2*y + k3 ; dz recomputed from (g, mask) exactly as in the reduce, or read (dz_in)
template <int DT>
__global__ __launch_bounds__(NT) void bn_bwd_apply_kernel(BwdArgs a, const void* __restrict__ dz_in,
                                                          const void* __restrict__ ysel,
                                                          const float* __restrict__ k1,
                                                          const float* __restrict__ k2,
                                                          const float* __restrict__ k3,
                                                          void* __restrict__ dy) {
  const long long n8 = a.rows * (a.C / 8);
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n8; i += (long long)gridDim.x * NT) {
    const long long row = i / (a.C / 8);
    const int c0 = (int)(i - row * (a.C / 8)) * 8;
    float dz[8], yv[8], y2v[8];
    if (dz_in) {
      load8<DT>(dz_in, (size_t)i * 8, dz);
    } else {
      make_dz<DT>(a, row, c0, dz, yv, y2v);
    }
    load8<DT>(ysel, (size_t)i * 8, yv);
    float A[8], B[8], Cc[8], o[8];
    ld8f(k1 + c0, A);
    ld8f(k2 + c0, B);
    ld8f(k3 + c0, Cc);
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = bnb_affine(A[e], B[e], Cc[e], dz[e], yv[e]);
    store8<DT>(dy, (size_t)i * 8, o);
  }
}

// dz read back (the common case: the consumer conv's dgrad epilogue stored it): pure stream,
// loop-invariant channel chunk (see bn_apply_kernel), packed math.
template <int DT>
__global__ __launch_bounds__(NT) void bn_bwd_apply_dz_kernel(const void* __restrict__ dz_in,
                                                             const void* __restrict__ ysel,
                                                             const float* __restrict__ k1,
                                                             const float* __restrict__ k2,
                                                             const float* __restrict__ k3,
                                                             void* __restrict__ dy, int n8, int C) {
  const int C8 = C >> 3;
  const int stride = gridDim.x * NT;
  const bool fixed = (stride % C8) == 0;
  f32x2 A[4], B[4], K3[4];
  int cprev = -1;
  for (int i = blockIdx.x * NT + threadIdx.x; i < n8; i += stride) {
    const int c0 = (i % C8) * 8;
    if (!fixed || cprev < 0) {
      ld8p<DT>(k1 + c0, A);
      ld8p<DT>(k2 + c0, B);
      ld8p<DT>(k3 + c0, K3);
      cprev = c0;
    }
    if constexpr (DT == DT_F32) {
      float dz[8], yv[8], o[8];
      load8<DT>(dz_in, (size_t)i * 8, dz);
      load8<DT>(ysel, (size_t)i * 8, yv);
#pragma unroll
      for (int e = 0; e < 8; ++e)
        o[e] = bnb_affine(A[e >> 1][e & 1], B[e >> 1][e & 1], K3[e >> 1][e & 1], dz[e], yv[e]);
      store8<DT>(dy, (size_t)i * 8, o);
      continue;
    }
    const i32x4 dz = reinterpret_cast<const i32x4*>(dz_in)[i];
    const i32x4 yv = reinterpret_cast<const i32x4*>(ysel)[i];
    i32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = (int)pack2<DT>(bnb_affine2(A[k], B[k], K3[k], unpack2<DT>((uint32_t)dz[k]),
                                        unpack2<DT>((uint32_t)yv[k])));
    reinterpret_cast<i32x4*>(dy)[i] = o;
  }
}

// 16-bit streaming forms with U independent 16-byte chunks per thread per trip: all U loads of
// both inputs are issued before the first use, so each lane keeps 2U (apply-dz) / up to 2U (apply)
// requests in flight instead of 2 -- the per-CU bytes in flight, not the instruction count, set
// a streaming kernel's HBM rate. The caller guarantees (stride % C8) == 0, so every chunk of a
// thread shares one channel octet: coefficients are loaded once. NTM bit 0: nontemporal loads,
// bit 1: nontemporal stores.
template <int NTL>
__device__ __forceinline__ i32x4 ldnt(const i32x4* p) {
  if constexpr (NTL) return __builtin_nontemporal_load(p);
  else return *p;
}

// 16-B output store of the streaming kernels by policy NTM: bit 2 = write-through (sc1: the line
// leaves the XCD's L2 with the store, so the kernel ends with no dirty output bytes to write back
// at its boundary -- MI355X_MICROARCH.md "stores of each flavour"), else bit 1 = nontemporal, else
// plain. ``rs``: buffer resource over the output (32-bit byte offsets; outputs < 2 GiB).
template <int NTM>
__device__ __forceinline__ void st_out(i32x4* base, __amdgpu_buffer_rsrc_t rs, int j, i32x4 o) {
  if constexpr (NTM & 4) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), rs, j * 16, 0, 16);
  else if constexpr (NTM & 2) __builtin_nontemporal_store(o, base + j);
  else base[j] = o;
}
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(void* p, int n8) {
  return __builtin_amdgcn_make_buffer_rsrc(p, (short)0, (int)((unsigned)n8 * 16u), 0x00020000);
}

template <int DT, int U, int NTM>
__global__ __launch_bounds__(NT) void bn_bwd_apply_dz_u_kernel(const void* __restrict__ dz_in,
                                                               const void* __restrict__ ysel,
                                                               const float* __restrict__ k1,
                                                               const float* __restrict__ k2,
                                                               const float* __restrict__ k3,
                                                               void* __restrict__ dy, int n8, int C) {
  const int C8 = C >> 3;
  const int stride = gridDim.x * NT;
  int i = blockIdx.x * NT + threadIdx.x;
  if (i >= n8) return;
  f32x2 A[4], B[4], K3[4];
  {
    const int c0 = (i % C8) * 8;
    ld8p<DT>(k1 + c0, A);
    ld8p<DT>(k2 + c0, B);
    ld8p<DT>(k3 + c0, K3);
  }
  const i32x4* dzp = reinterpret_cast<const i32x4*>(dz_in);
  const i32x4* yp = reinterpret_cast<const i32x4*>(ysel);
  i32x4* op = reinterpret_cast<i32x4*>(dy);
  const __amdgpu_buffer_rsrc_t rs = out_rsrc(dy, n8);
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    i32x4 dz[U], yv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dz[u] = ldnt<NTM & 1>(dzp + i + u * stride);
      yv[u] = ldnt<NTM & 1>(yp + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      i32x4 o;
#pragma unroll
      for (int k = 0; k < 4; ++k)
        o[k] = (int)pack2<DT>(bnb_affine2(A[k], B[k], K3[k], unpack2<DT>((uint32_t)dz[u][k]),
                                          unpack2<DT>((uint32_t)yv[u][k])));
      st_out<NTM>(op, rs, i + u * stride, o);
    }
  }
  for (; i < n8; i += stride) {
    const i32x4 dz = dzp[i], yv = yp[i];
    i32x4 o;
#pragma unroll
    for (int k = 0; k < 4; ++k)
      o[k] = (int)pack2<DT>(bnb_affine2(A[k], B[k], K3[k], unpack2<DT>((uint32_t)dz[k]),
                                        unpack2<DT>((uint32_t)yv[k])));
    op[i] = o;
  }
}

// Both branches of a downsample block's tail in one pass: dz (the masked gradient of
// relu(bn(y) + bn2(y2))) is read ONCE for dy = k[0..3C)(dz, y) and dy2 = k[3C..6C)(dz, y2) --
// 3 reads + 2 writes per chunk instead of 4 + 2 over two launches. U chunks per trip as above.
template <int DT, int U, int NTM>
__global__ __launch_bounds__(NT) void bn_bwd_apply_dz2_u_kernel(const void* __restrict__ dz_in,
                                                                const void* __restrict__ ysel,
                                                                const void* __restrict__ y2sel,
                                                                const float* __restrict__ k,
                                                                void* __restrict__ dy,
                                                                void* __restrict__ dy2, int n8, int C) {
  const int C8 = C >> 3;
  const int stride = gridDim.x * NT;
  int i = blockIdx.x * NT + threadIdx.x;
  if (i >= n8) return;
  f32x2 A[4], B[4], K3[4], A2[4], B2[4], K32[4];
  {
    const int c0 = (i % C8) * 8;
    ld8p<DT>(k + c0, A);
    ld8p<DT>(k + C + c0, B);
    ld8p<DT>(k + 2 * C + c0, K3);
    ld8p<DT>(k + 3 * C + c0, A2);
    ld8p<DT>(k + 4 * C + c0, B2);
    ld8p<DT>(k + 5 * C + c0, K32);
  }
  const i32x4* dzp = reinterpret_cast<const i32x4*>(dz_in);
  const i32x4* yp = reinterpret_cast<const i32x4*>(ysel);
  const i32x4* y2p = reinterpret_cast<const i32x4*>(y2sel);
  i32x4* op = reinterpret_cast<i32x4*>(dy);
  i32x4* op2 = reinterpret_cast<i32x4*>(dy2);
  const __amdgpu_buffer_rsrc_t rs = out_rsrc(dy, n8), rs2 = out_rsrc(dy2, n8);
  auto one = [&](const i32x4& dz, const i32x4& yv, const i32x4& y2v, int j) __attribute__((always_inline)) {
    i32x4 o, o2;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const f32x2 d = unpack2<DT>((uint32_t)dz[q]);
      o[q] = (int)pack2<DT>(bnb_affine2(A[q], B[q], K3[q], d, unpack2<DT>((uint32_t)yv[q])));
      o2[q] = (int)pack2<DT>(bnb_affine2(A2[q], B2[q], K32[q], d, unpack2<DT>((uint32_t)y2v[q])));
    }
    st_out<NTM>(op, rs, j, o);
    st_out<NTM>(op2, rs2, j, o2);
  };
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    i32x4 dz[U], yv[U], y2v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      dz[u] = ldnt<NTM & 1>(dzp + i + u * stride);
      yv[u] = ldnt<NTM & 1>(yp + i + u * stride);
      y2v[u] = ldnt<NTM & 1>(y2p + i + u * stride);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(dz[u], yv[u], y2v[u], i + u * stride);
  }
  for (; i < n8; i += stride) one(dzp[i], yp[i], y2p[i], i);
}

// bn_apply_kernel's 16-bit path with U chunks per trip (see bn_bwd_apply_dz_u_kernel).
template <int DT, int U, int NTM>
__global__ __launch_bounds__(NT) void bn_apply_u_kernel(
    const void* __restrict__ y, const float* __restrict__ sc, const float* __restrict__ sh,
    const void* __restrict__ r2, const float* __restrict__ sc2, const float* __restrict__ sh2,
    void* __restrict__ out, int n8, int C, int mode, int relu, uint8_t* __restrict__ mask) {
  const int C8 = C >> 3;
  const int stride = gridDim.x * NT;
  int i = blockIdx.x * NT + threadIdx.x;
  if (i >= n8) return;
  f32x2 a[4], b[4], a2[4], b2[4];
  {
    const int c0 = (i % C8) * 8;
    ld8p<DT>(sc + c0, a);
    ld8p<DT>(sh + c0, b);
    if (mode == 2) {
      ld8p<DT>(sc2 + c0, a2);
      ld8p<DT>(sh2 + c0, b2);
    }
  }
  const i32x4* yp = reinterpret_cast<const i32x4*>(y);
  const i32x4* rp = reinterpret_cast<const i32x4*>(r2);
  i32x4* op = reinterpret_cast<i32x4*>(out);
  const __amdgpu_buffer_rsrc_t rs = out_rsrc(out, n8);
  auto one = [&](const i32x4& yv, const i32x4& rv, int j) {
    i32x4 o;
    uint32_t bits = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      f32x2 v = tail_pre2(unpack2<DT>((uint32_t)yv[k]), a[k], b[k], unpack2<DT>((uint32_t)rv[k]),
                          a2[k], b2[k], mode);
      if (relu) v = f32x2{fmaxf(v.x, 0.f), fmaxf(v.y, 0.f)};
      o[k] = (int)pack2<DT>(v);
      bits |= (v.x > 0.f ? 1u : 0u) << (2 * k);
      bits |= (v.y > 0.f ? 1u : 0u) << (2 * k + 1);
    }
    st_out<NTM>(op, rs, j, o);
    if (mask) mask[j] = (uint8_t)bits;
  };
  for (; i + (U - 1) * stride < n8; i += U * stride) {
    i32x4 yv[U], rv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      yv[u] = ldnt<NTM & 1>(yp + i + u * stride);
      rv[u] = mode ? ldnt<NTM & 1>(rp + i + u * stride) : i32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) one(yv[u], rv[u], i + u * stride);
  }
  for (; i < n8; i += stride) one(yp[i], mode ? rp[i] : i32x4{0, 0, 0, 0}, i);
}

// first stage of the statistics reduction: [G][QC] partial slabs -> [S][QC] (S << G), coalesced
__global__ __launch_bounds__(256) void slab_reduce_kernel(const float* __restrict__ in, int G, int QC,
                                                          int rows_per, float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= QC) return;
  const int g0 = blockIdx.y * rows_per;
  const int g1 = min(G, g0 + rows_per);
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  int g = g0;
  for (; g + 3 < g1; g += 4) {
    s0 += in[(size_t)g * QC + c];
    s1 += in[(size_t)(g + 1) * QC + c];
    s2 += in[(size_t)(g + 2) * QC + c];
    s3 += in[(size_t)(g + 3) * QC + c];
  }
  for (; g < g1; ++g) s0 += in[(size_t)g * QC + c];
  out[(size_t)blockIdx.y * QC + c] = (s0 + s1) + (s2 + s3);
}

inline int grid_for(long long n, int cap = 8192) {
  long long b = (n + NT - 1) / NT;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

// Streaming-kernel shape for the 16-bit apply passes: chunks per thread per trip (0 = the plain
// one-chunk kernels), memory policy (bit 0 nontemporal loads, bit 1 nontemporal stores, bit 2
// write-through stores -- 4-chunk launches: 4..7 run as 5), grid cap in blocks.
// unroll < 0 (auto): tensors of at least min_mb MiB (the host passes 50: in-step best of
// 30-200, ext.stream_cfg) take -unroll chunks (-1: 4), nontemporal policy ntm and grid cap
// (host default: nt loads + stores, 65536); smaller ones the one-chunk kernels
// (tools/stream_bench.py, profiles/stream_bench_r2.txt: isolated -11 % on the >= 160 MB passes).
struct StreamCfg {
  int unroll, ntm, cap, min_mb;
};
StreamCfg g_stream{0, 0, 8192, 100};

// Launch KER<DT, U, NTM> for the configured (U, NTM); false when the shape does not qualify.
#define STREAM_DISPATCH(KER, DT, g, st, ...)                                              \
  STREAM_DISPATCH_UM(KER, DT, g, st, stream_chunks(), g_stream.ntm, __VA_ARGS__)
#define STREAM_DISPATCH_UM(KER, DT, g, st, U_, M_, ...)                                    \
  do {                                                                                        \
    const int u_ = (U_), m_ = (M_);                                                           \
    if (u_ == 2 && m_ == 0) TRACKED_LAUNCH((KER<DT, 2, 0>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 2 && m_ == 1) TRACKED_LAUNCH((KER<DT, 2, 1>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 2 && m_ == 2) TRACKED_LAUNCH((KER<DT, 2, 2>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 2) TRACKED_LAUNCH((KER<DT, 2, 3>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 4 && m_ == 0) TRACKED_LAUNCH((KER<DT, 4, 0>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 4 && m_ == 1) TRACKED_LAUNCH((KER<DT, 4, 1>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 4 && m_ == 2) TRACKED_LAUNCH((KER<DT, 4, 2>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 4 && m_ >= 4) TRACKED_LAUNCH((KER<DT, 4, 5>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (u_ == 4) TRACKED_LAUNCH((KER<DT, 4, 3>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (m_ == 0) TRACKED_LAUNCH((KER<DT, 1, 0>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (m_ == 1) TRACKED_LAUNCH((KER<DT, 1, 1>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else if (m_ == 2) TRACKED_LAUNCH((KER<DT, 1, 2>), dim3(g), dim3(NT), 0, st, __VA_ARGS__); \
    else TRACKED_LAUNCH((KER<DT, 1, 3>), dim3(g), dim3(NT), 0, st, __VA_ARGS__);         \
  } while (0)

// chunks per thread per trip: unroll > 0 as given; auto (unroll < 0): -unroll, -1 meaning 4
inline int stream_chunks() {
  return g_stream.unroll > 0 ? g_stream.unroll : (g_stream.unroll == -1 ? 4 : -g_stream.unroll);
}

// grid for the U-chunk kernels: ~n8/U threads, capped; 0 when a thread's chunks would not share
// one channel octet (stride % C8 != 0)
inline int stream_grid(long long n8, int C) {
  if (g_stream.unroll == 0) return 0;
  const bool autoc = g_stream.unroll < 0;
  if (autoc && n8 * 16 < ((long long)g_stream.min_mb << 20)) return 0;
  const int u = stream_chunks();
  const int g = grid_for((n8 + u - 1) / u, g_stream.cap);
  return ((long long)g * NT) % (C >> 3) == 0 ? g : 0;
}

}  // namespace

extern "C" {

// Streaming apply kernels (see StreamCfg): unroll < 0 = auto with -unroll chunks (-1: 4) for
// tensors >= min_mb MiB, 0 = the one-chunk kernels, 1/2/4 = that many chunks for every shape;
// ntm / cap apply to the multi-chunk launches. Returns the previous unroll.
int pda_set_stream_cfg(int unroll, int ntm, int cap, int min_mb) {
  const int prev = g_stream.unroll;
  const int a = unroll < 0 ? -unroll : unroll;
  g_stream.unroll = (a == 1 || a == 2 || a == 4) ? unroll : 0;
  g_stream.ntm = ntm & 7;
  g_stream.cap = cap > 0 ? cap : 8192;
  g_stream.min_mb = min_mb >= 0 ? min_mb : 100;
  return prev;
}

int pda_slab_reduce(const float* in, int G, int QC, int S, float* out, hipStream_t st) {
  const int rows_per = (G + S - 1) / S;
  const int s = (G + rows_per - 1) / rows_per;
  TRACKED_LAUNCH(slab_reduce_kernel, dim3((QC + 255) / 256, s), dim3(256), 0, st, in, G, QC, rows_per,
                     out);
  return (int)hipGetLastError() ? -1 : s;
}

int pda_bn_finalize_tot(const double* tot, int C, double count, const float* gamma,
                        const float* beta, float eps, float momentum, float* mean, float* invstd,
                        float* scale, float* shift, float* rmean, float* rvar, long long* nbt,
                        int update_running, hipStream_t st) {
  TRACKED_LAUNCH(bn_finalize_tot_kernel, dim3((C + 255) / 256), dim3(256), 0, st, tot, C, count,
                     gamma, beta, eps, momentum, mean, invstd, scale, shift, rmean, rvar, nbt,
                     update_running);
  return (int)hipGetLastError();
}

// Partial statistics -> BatchNorm coefficients in one launch (bn_stats_kernel). slabs: f64 >=
// S * nq * C; cnt: int32 >= ceil(C / 256), zero (and left zero). Returns -2 on a bad shape.
// cg: channels per block group (a power of two in [4, 256]; 0 = 256). Fewer channels per group
// give each channel quad more lanes (SL = 1024 / cg): shorter serial chains in both levels.
static int stats_cg(int C, int cg) {
  if (cg <= 0 || cg > 256 || (cg & (cg - 1)) || cg < 4) cg = 256;
  return C < cg ? C : cg;
}

int pda_bn_fwd_stats(const float* part, int T, int C, int bm, int M, int S, double* slabs, int* cnt,
                     const BnFwdOut* o, int cg, hipStream_t st) {
  if ((C & 3) || S <= 0 || S > T || !o || !cnt || !slabs) return -2;
  const int CG = stats_cg(C, cg);   // (a ragged last group: its lanes past C stay idle)
  TRACKED_LAUNCH((bn_stats_kernel<0, 2, BnFwdOut>), dim3(S, (C + CG - 1) / CG), dim3(256), 0, st,
                     part, T, C, bm, M, CG, slabs, cnt, *o);
  return (int)hipGetLastError();
}

int pda_bn_bwd_stats(const float* part, int T, int nq, int C, int S, double* slabs, int* cnt,
                     const BnBwdOut* o, int cg, hipStream_t st) {
  if ((C & 3) || S <= 0 || S > T || !o || !cnt || !slabs || !o->k || (nq != 2 && nq != 3))
    return -2;
  const int CG = stats_cg(C, cg);   // (a ragged last group: its lanes past C stay idle)
  const dim3 grid(S, (C + CG - 1) / CG);
  if (nq == 2)
    TRACKED_LAUNCH((bn_stats_kernel<1, 2, BnBwdOut>), grid, dim3(256), 0, st, part, T, C, 0, 0, CG,
                       slabs, cnt, *o);
  else
    TRACKED_LAUNCH((bn_stats_kernel<1, 3, BnBwdOut>), grid, dim3(256), 0, st, part, T, C, 0, 0, CG,
                       slabs, cnt, *o);
  return (int)hipGetLastError();
}

int pda_bn_eval_coeffs(const float* gamma, const float* beta, const float* rm, const float* rv,
                       float eps, int C, float* scale, float* shift, hipStream_t st) {
  TRACKED_LAUNCH(bn_eval_coeffs_kernel, dim3((C + 255) / 256), dim3(256), 0, st, gamma, beta, rm,
                     rv, eps, C, scale, shift);
  return (int)hipGetLastError();
}

static FastDiv make_div(uint32_t d) {
  FastDiv f;
  f.d = d;
  uint32_t s = 0;
  while ((1ull << s) < d) ++s;
  f.s = s;
  f.m = (uint32_t)(((1ull << 32) * ((1ull << s) - d)) / d + 1);
  return f;
}

// mask (nullable): one byte per 8 elements, bit e = (output element e > 0) -- lets the backward of an
// identity-shortcut tail skip re-reading the residual to rebuild its ReLU mask
int pda_bn_apply(const void* y, const float* sc, const float* sh, const void* r2, const float* sc2,
                 const float* sh2, void* out, long long numel, int C, int mode, int relu,
                 void* mask, int dt, hipStream_t st) {
  if (numel / 8 >= (1ll << 31)) return -2;
  const int n8 = (int)(numel / 8);
  const int g = grid_for(n8);
#define ARGS (const void*)y, sc, sh, (const void*)r2, sc2, sh2, (void*)out, n8, C, mode, relu, \
             (uint8_t*)mask
  if (g_stream.unroll != 0 && dt != DT_F32 && (C & 7) == 0) {
    const int gs = stream_grid(n8, C);
    if (gs > 0) {
      if (dt == DT_BF16) STREAM_DISPATCH(bn_apply_u_kernel, DT_BF16, gs, st, ARGS);
      else STREAM_DISPATCH(bn_apply_u_kernel, DT_F16, gs, st, ARGS);
      return (int)hipGetLastError();
    }
  }
  if (dt == DT_BF16) TRACKED_LAUNCH(bn_apply_kernel<DT_BF16>, dim3(g), dim3(NT), 0, st, ARGS);
  else if (dt == DT_F32) TRACKED_LAUNCH(bn_apply_kernel<DT_F32>, dim3(g), dim3(NT), 0, st, ARGS);
  else TRACKED_LAUNCH(bn_apply_kernel<DT_F16>, dim3(g), dim3(NT), 0, st, ARGS);
#undef ARGS
  return (int)hipGetLastError();
}

int pda_stem_pool(const void* y, const float* sc, const float* sh, void* out, void* arg, int N,
                  int H, int W, int C, int Ho, int Wo, int dt, hipStream_t st) {
  if ((long long)N * H * W * (C / 8) >= (1ll << 31)) return -2;
  const int g = grid_for((long long)N * Ho * Wo * (C / 8));
  const char* rv = pda_reverse_env();
  const int rev = (rv && strstr(rv, "stem_pool")) ? 1 : 0;
#define ARGS (const void*)y, sc, sh, (void*)out, (uint8_t*)arg, N, H, W, C, Ho, Wo, make_div(C / 8), \
             make_div(Wo), make_div(Ho), rev
  if (dt == DT_BF16) TRACKED_LAUNCH(stem_pool_kernel<DT_BF16>, dim3(g), dim3(NT), 0, st, ARGS);
  else if (dt == DT_F32) TRACKED_LAUNCH(stem_pool_kernel<DT_F32>, dim3(g), dim3(NT), 0, st, ARGS);
  else TRACKED_LAUNCH(stem_pool_kernel<DT_F16>, dim3(g), dim3(NT), 0, st, ARGS);
#undef ARGS
  return (int)hipGetLastError();
}

int pda_maxpool_bwd(const void* dout, const void* dout2, const void* arg, void* din, int N, int H,
                    int W, int C, int Ho, int Wo, int dt, hipStream_t st) {
  if ((long long)N * H * W * (C / 8) >= (1ll << 31)) return -2;
  const int g = grid_for((long long)N * H * W * (C / 8));
#define ARGS (const void*)dout, (const void*)dout2, (const uint8_t*)arg, (void*)din, N, H, W, C, Ho, Wo, \
             make_div(C / 8), make_div(W), make_div(H)
  if (dt == DT_BF16) TRACKED_LAUNCH(maxpool_bwd_kernel<DT_BF16>, dim3(g), dim3(NT), 0, st, ARGS);
  else if (dt == DT_F32) TRACKED_LAUNCH(maxpool_bwd_kernel<DT_F32>, dim3(g), dim3(NT), 0, st, ARGS);
  else TRACKED_LAUNCH(maxpool_bwd_kernel<DT_F16>, dim3(g), dim3(NT), 0, st, ARGS);
#undef ARGS
  return (int)hipGetLastError();
}

int pda_tail_pool(const void* y, const float* sc, const float* sh, const void* r2, const float* sc2,
                  const float* sh2, void* out, int N, int HW, int C, int mode, int dt,
                  hipStream_t st) {
#define ARGS (const void*)y, sc, sh, (const void*)r2, sc2, sh2, (void*)out, HW, C, mode
  if (dt == DT_BF16) TRACKED_LAUNCH(tail_pool_kernel<DT_BF16>, dim3(N), dim3(NT), 0, st, ARGS);
  else if (dt == DT_F32) TRACKED_LAUNCH(tail_pool_kernel<DT_F32>, dim3(N), dim3(NT), 0, st, ARGS);
  else TRACKED_LAUNCH(tail_pool_kernel<DT_F16>, dim3(N), dim3(NT), 0, st, ARGS);
#undef ARGS
  return (int)hipGetLastError();
}

struct BwdArgsC {  // mirrors ops/ext.py
  const void* g1; const void* g2; const void* gp; int HW;
  const void* y; const float* sc; const float* sh;
  const void* y2; const float* sc2; const float* sh2;
  int mode; void* dz_out;
  float* part; int nq; long long rows; int C;
};

static BwdArgs to_args(const BwdArgsC* c) {
  BwdArgs a;
  a.g1 = (const void*)c->g1; a.g2 = (const void*)c->g2; a.gp = (const void*)c->gp; a.HW = c->HW;
  a.y = (const void*)c->y; a.sc = c->sc; a.sh = c->sh;
  a.y2 = (const void*)c->y2; a.sc2 = c->sc2; a.sh2 = c->sh2;
  a.mode = c->mode; a.dz_out = (void*)c->dz_out;
  a.part = c->part; a.nq = c->nq; a.rows = c->rows; a.C = c->C; a.rows_per_block = 0;
  return a;
}

// G = number of partial slabs written (returned through *G_out); part must hold G*nq*C floats.
int pda_bn_bwd_reduce(const BwdArgsC* c, int G, int dt, hipStream_t st) {
  BwdArgs a = to_args(c);
  a.rows_per_block = (a.rows + G - 1) / G;
#define K(D) TRACKED_LAUNCH(bn_bwd_reduce_kernel<D>, dim3(G), dim3(NT), 0, st, a)
  if (dt == DT_BF16) K(DT_BF16); else if (dt == DT_F32) K(DT_F32); else K(DT_F16);
#undef K
  return (int)hipGetLastError();
}

// stem backward reduce (maxpool gather + ReLU mask + dz store + partials [G][2][C])
int pda_stem_bwd_reduce(const void* dout, const void* dout2, const void* arg, const void* y,
                        const float* sc, const float* sh, void* dz_out, float* part, int G, int N,
                        int H, int W, int C, int Ho, int Wo, int dt, hipStream_t st) {
  const long long rows = (long long)N * H * W;
  // the quad decomposition assumes the 3x3/2 pad-1 pooling geometry
  if (rows * C >= (1ll << 31) || C % 8 || Ho != (H + 1) / 2 || Wo != (W + 1) / 2) return -2;
  const long long quads = (long long)N * Ho * Wo;
  const long long qpb = (quads + G - 1) / G;
#define K(D) TRACKED_LAUNCH(stem_bwd_reduce_kernel<D>, dim3(G), dim3(NT), 0, st, (const void*)dout, \
                                (const void*)dout2, (const uint8_t*)arg, (const void*)y, sc, sh,       \
                                (void*)dz_out, part, quads, qpb, H, W, C, Ho, Wo, make_div(Wo),        \
                                make_div(Ho))
  if (dt == DT_BF16) K(DT_BF16); else if (dt == DT_F32) K(DT_F32); else K(DT_F16);
#undef K
  return (int)hipGetLastError();
}

int pda_bn_bwd_finalize(const float* part, int G, int nq, int qy, int C, float count,
                        const float* gamma, const float* mean, const float* invstd, float* dgamma,
                        float* dbeta, float* k1, float* k2, float* k3, float gscale, int accumulate,
                        hipStream_t st) {
  TRACKED_LAUNCH(bn_bwd_finalize_kernel, dim3((C + 15) / 16), dim3(1024), 0, st, part, G, nq, qy,
                     C, count, gamma, mean, invstd, dgamma, dbeta, k1, k2, k3, gscale, accumulate);
  return (int)hipGetLastError();
}

// Both branches of a downsample tail in one pass (16-bit; -1 for other dtypes): k = [2][3][C].
int pda_bn_bwd_apply2(const void* dz, const void* y, const void* y2, const float* k, void* dy,
                      void* dy2, long long rows, int C, int dt, hipStream_t st) {
  if ((dt != DT_BF16 && dt != DT_F16) || (C & 7) || rows * (C / 8) >= (1ll << 31)) return -1;
  const int n8 = (int)(rows * (C / 8));
  // streaming config as the one-branch pass (auto: 4 chunks + nontemporal for >= 100 MiB),
  // else one chunk per trip
  int gs = stream_grid(n8, C);
  int u = stream_chunks(), m = g_stream.ntm;
  if (gs <= 0) {
    gs = grid_for(n8);
    if (((long long)gs * NT) % (C >> 3)) return -1;
    u = 1;
    m = 0;
  }
#define KA dz, y, y2, k, dy, dy2, n8, C
  if (dt == DT_BF16) STREAM_DISPATCH_UM(bn_bwd_apply_dz2_u_kernel, DT_BF16, gs, st, u, m, KA);
  else STREAM_DISPATCH_UM(bn_bwd_apply_dz2_u_kernel, DT_F16, gs, st, u, m, KA);
#undef KA
  return (int)hipGetLastError();
}

int pda_bn_bwd_apply(const BwdArgsC* c, const void* dz_in, const void* ysel, const float* k1,
                     const float* k2, const float* k3, void* dy, int dt, hipStream_t st) {
  BwdArgs a = to_args(c);
  const int g = grid_for(a.rows * (a.C / 8));
  if (dz_in && a.rows * (a.C / 8) < (1ll << 31)) {
    const int n8 = (int)(a.rows * (a.C / 8));
    const int gs = dt != DT_F32 ? stream_grid(n8, a.C) : 0;
    if (gs > 0) {
#define KA (const void*)dz_in, (const void*)ysel, k1, k2, k3, (void*)dy, n8, a.C
      if (dt == DT_BF16) STREAM_DISPATCH(bn_bwd_apply_dz_u_kernel, DT_BF16, gs, st, KA);
      else STREAM_DISPATCH(bn_bwd_apply_dz_u_kernel, DT_F16, gs, st, KA);
#undef KA
      return (int)hipGetLastError();
    }
#define K(D) TRACKED_LAUNCH(bn_bwd_apply_dz_kernel<D>, dim3(g), dim3(NT), 0, st, (const void*)dz_in, \
                                (const void*)ysel, k1, k2, k3, (void*)dy, n8, a.C)
    if (dt == DT_BF16) K(DT_BF16); else if (dt == DT_F32) K(DT_F32); else K(DT_F16);
#undef K
    return (int)hipGetLastError();
  }
#define K(D) TRACKED_LAUNCH(bn_bwd_apply_kernel<D>, dim3(g), dim3(NT), 0, st, a, (const void*)dz_in, \
                                (const void*)ysel, k1, k2, k3, (void*)dy)
  if (dt == DT_BF16) K(DT_BF16); else if (dt == DT_F32) K(DT_F32); else K(DT_F16);
#undef K
  return (int)hipGetLastError();
}

}  // extern "C"
