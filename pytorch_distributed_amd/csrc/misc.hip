// Loss, optimizer, AMP and data kernels for gfx950.
//
//   xent_fwd_bwd   : log-softmax + NLL (mean) forward AND its gradient in one pass, one wave per row
//                    of the [B, classes] f32 logits (replaces ATen log_softmax/nll_loss fwd+bwd, K8);
//                    dlogits written 16-bit into a zero-padded [B, ld] buffer for the fc dgrad/wgrad
//   topk_acc       : top-1 / top-5 hit counters (replaces topk/eq/sum of validate, K11)
//   col_sum        : sum over rows of a 16-bit [rows, C] matrix (fc bias gradient)
//   sgd_flat       : ONE launch over the whole flat parameter buffer: AMP unscale, weight decay,
//                    momentum (torch SGD semantics, first step buf = d_p), update, 16-bit shadow
//                    write; skipped on device when found_inf (no host sync) (K9, K10)
//   amp_scan : non-finite scan of the flat gradient + GradScaler state machine (one launch)
//   pack_stem      : f32 master [64][7][7][3] -> 16-bit [64][448] (taps x 8 padded channels)
//   synth_nhwc8    : on-device synthetic ImageNet batch: NHWC, 3 channels padded to 8, 16-bit,
//                    bit-compatible with data/synthetic.py (label + uniform u) (K12)
//   nchw_to_nhwc8  : any f32 NCHW image batch -> NHWC8 16-bit model input
#include "common.h"

namespace {

constexpr int NT = 256;

// ------------------------------------------------------------------ softmax cross-entropy
__global__ __launch_bounds__(NT) void xent_kernel(const float* __restrict__ logits, int B, int K,
                                                  int ld_in, const long long* __restrict__ labels,
                                                  float* __restrict__ loss_rows, void* __restrict__ dlog,
                                                  int ld_out, float gscale, const float* __restrict__ gdev, int dt,
                                                  int want_grad) {
  const int wave = (blockIdx.x * NT + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= B) return;
  const float* x = logits + (size_t)wave * ld_in;
  float m = -INFINITY;
  for (int k = lane; k < K; k += 64) m = fmaxf(m, x[k]);
  m = wave_max(m);
  float s = 0.f;
  for (int k = lane; k < K; k += 64) s += __expf(x[k] - m);
  s = wave_sum(s);
  const float lse = m + __logf(s);
  const int lab = (int)labels[wave];
  if (lane == 0) loss_rows[wave] = lse - x[lab];
  if (!want_grad) return;
  const float inv = 1.f / s;
  if (gdev) gscale *= gdev[0];
  const size_t drow = (size_t)wave * ld_out;
  for (int k = lane; k < ld_out; k += 64) {
    float g = 0.f;
    if (k < K) g = (__expf(x[k] - m) * inv - (k == lab ? 1.f : 0.f)) * gscale;
    st_any(dlog, drow + k, g, dt);
  }
}

// loss = mean(loss_rows) (deterministic single block)
__global__ __launch_bounds__(1024) void mean_kernel(const float* __restrict__ v, int n,
                                                    float* __restrict__ out) {
  __shared__ float red[16];
  float s = 0.f;
  for (int i = threadIdx.x; i < n; i += 1024) s += v[i];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < 16; ++i) t += red[i];
    out[0] = t / (float)n;
  }
}

// top-1/top-5 hits: out[0] += top1 hits, out[1] += top5 hits (ties broken like torch.topk: lower idx)
__global__ __launch_bounds__(NT) void topk_kernel(const float* __restrict__ logits, int B, int K,
                                                  int ld, const long long* __restrict__ labels,
                                                  float* __restrict__ hits) {
  const int wave = (blockIdx.x * NT + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= B) return;
  const float* x = logits + (size_t)wave * ld;
  const int lab = (int)labels[wave];
  const float v = x[lab];
  // rank = number of classes strictly better than the label (ties: lower index first)
  int better = 0;
  for (int k = lane; k < K; k += 64) {
    const float u = x[k];
    better += (u > v || (u == v && k < lab)) ? 1 : 0;
  }
  for (int o = 32; o > 0; o >>= 1) better += __shfl_xor(better, o, 64);
  if (lane == 0) {
    if (better < 1) atomicAdd(&hits[0], 1.f);
    if (better < 5) atomicAdd(&hits[1], 1.f);
  }
}

// out[c] = scale * sum_r x[r][c]  (x: 16-bit [rows][ld]). Block = 64 columns x 16 row slices
// (1024 threads): each thread sums every 16th row of its column (independent loads, pipelined),
// then a fixed-order LDS combine -- deterministic, no serial 400-load chain per column.
__global__ __launch_bounds__(1024) void col_sum_kernel(const void* __restrict__ x, int rows, int C,
                                                       int ld, float scale, float* __restrict__ out,
                                                       int dt, int accumulate) {
  __shared__ float red[16][64];
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  float s = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int r = sl; r < rows; r += 16) {
      s += ld_any(x, (size_t)r * ld + c, dt);
    }
  }
  red[sl][cl] = s;
  __syncthreads();
  if (sl == 0 && c < C) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) t += red[k][cl];
    out[c] = t * scale + (accumulate ? out[c] : 0.f);
  }
}

// ------------------------------------------------------------------ optimizer
// flags: bit0 = momentum buffer initialised (else buf = d_p), bit1 = write shadow
__global__ __launch_bounds__(NT) void sgd_flat_kernel(float* __restrict__ p, float* __restrict__ g,
                                                      float* __restrict__ buf, u16* __restrict__ shadow,
                                                      long long n, float lr, float momentum,
                                                      float wd, const float* __restrict__ inv_scale_src,
                                                      const float* __restrict__ found_inf, int flags,
                                                      int dt) {
  if (found_inf && found_inf[0] != 0.f) return;
  const float inv = inv_scale_src ? inv_scale_src[0] : 1.f;   // published by amp_scan_kernel
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n4; i += (long long)gridDim.x * NT) {
    f32x4 pv = reinterpret_cast<f32x4*>(p)[i];
    f32x4 gv = reinterpret_cast<f32x4*>(g)[i];
    f32x4 bv = reinterpret_cast<f32x4*>(buf)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float d = gv[e] * inv + wd * pv[e];
      float b = (flags & 1) ? momentum * bv[e] + d : d;
      bv[e] = b;
      pv[e] -= lr * b;
    }
    reinterpret_cast<f32x4*>(p)[i] = pv;
    reinterpret_cast<f32x4*>(buf)[i] = bv;
    if (flags & 2) {
      u16 h[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) h[e] = dt == DT_BF16 ? f32_to_bf16(pv[e]) : f32_to_f16(pv[e]);
      reinterpret_cast<uint2*>(shadow)[i] = *reinterpret_cast<uint2*>(h);
    }
  }
  // tail (n % 4)
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) {
    const long long i = (n4 << 2) + threadIdx.x;
    float d = g[i] * inv + wd * p[i];
    float b = (flags & 1) ? momentum * buf[i] + d : d;
    buf[i] = b;
    p[i] -= lr * b;
    if (flags & 2) shadow[i] = dt == DT_BF16 ? f32_to_bf16(p[i]) : f32_to_f16(p[i]);
  }
}

__global__ __launch_bounds__(NT) void cast_flat_kernel(const float* __restrict__ p, u16* __restrict__ s,
                                                       long long n, int dt) {
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n; i += (long long)gridDim.x * NT)
    s[i] = dt == DT_BF16 ? f32_to_bf16(p[i]) : f32_to_f16(p[i]);
}

// AMP (GradScaler) in ONE launch before the fused SGD: non-finite scan of the flat gradient, and
// the LAST workgroup to finish (arrival counter, agent-scope acq_rel) publishes
//   found_inf[0] = any non-finite in g,  inv[0] = 1/scale (what the SGD unscales by),
// then applies torch._amp_update_scale_ to scale/tracker (skipped when tracker == nullptr).
// ws[0..1] = one 64-bit word (arrivals | non-finite blocks << 32), reset by that last workgroup,
// so the kernel needs no memset and replays inside a HIP graph.
__global__ __launch_bounds__(NT) void amp_scan_kernel(const float* __restrict__ g, long long n,
                                                      float* __restrict__ found_inf,
                                                      float* __restrict__ inv,
                                                      float* __restrict__ scale,
                                                      int* __restrict__ tracker, int* ws,
                                                      float growth, float backoff, int interval) {
  __shared__ int s_bad, s_last;
  if (threadIdx.x == 0) s_bad = 0;
  bool bad = false;
  const long long n4 = n >> 2;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < n4; i += (long long)gridDim.x * NT) {
    const f32x4 v = reinterpret_cast<const f32x4*>(g)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) bad |= !(fabsf(v[e]) <= 3.4028235e38f);
  }
  if (blockIdx.x == 0 && threadIdx.x < (n & 3)) bad |= !(fabsf(g[(n4 << 2) + threadIdx.x]) <= 3.4028235e38f);
  __syncthreads();
  if (__any(bad) && (threadIdx.x & 63) == 0) s_bad = 1;
  __syncthreads();
  // ONE relaxed 64-bit arrival per block carries its payload: low word = arrivals, high word =
  // blocks that saw a non-finite value. The last arriver's fetch result (+ its own add) holds every
  // block's flag, so no release / acquire fences (each an L2 writeback / invalidate) are needed.
  __shared__ int s_any;
  if (threadIdx.x == 0) {
    const unsigned long long add = 1ull + (s_bad ? (1ull << 32) : 0ull);
    const unsigned long long prev = __hip_atomic_fetch_add(
        reinterpret_cast<unsigned long long*>(ws), add, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = (unsigned)(prev & 0xffffffffull) == gridDim.x - 1;
    s_any = ((prev + add) >> 32) != 0;
  }
  __syncthreads();
  if (s_last && threadIdx.x == 0) {
    const bool f = s_any != 0;
    const float sc = scale[0];
    found_inf[0] = f ? 1.f : 0.f;
    inv[0] = (float)(1.0 / (double)sc);
    if (tracker) {
      if (f) {
        scale[0] = sc * backoff;
        tracker[0] = 0;
      } else {
        const int t = tracker[0] + 1;
        if (t == interval) {
          const float ns = sc * growth;
          if (fabsf(ns) <= 3.4028235e38f) scale[0] = ns;
          tracker[0] = 0;
        } else {
          tracker[0] = t;
        }
      }
    }
    __hip_atomic_store(reinterpret_cast<unsigned long long*>(ws), 0ull, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  }
}

// stem weight pack: src f32 [Cout][R*S][Cin] (channels-last OHWI) -> dst 16-bit [Cout][Kpad]
__global__ void pack_stem_kernel(const float* __restrict__ src, void* __restrict__ dst, int Cout,
                                 int RS, int Cin, int Cpad, int Kpad, int dt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Cout * Kpad) return;
  const int co = i / Kpad, k = i - co * Kpad;
  const int tap = k / Cpad, c = k - tap * Cpad;
  float v = 0.f;
  if (tap < RS && c < Cin) v = src[((size_t)co * RS + tap) * Cin + c];
  st_any(dst, i, v, dt);
}

// ------------------------------------------------------------------ data
__device__ __forceinline__ uint32_t hash32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7FEB352Du;
  x ^= x >> 15;
  x *= 0x846CA68Bu;
  x ^= x >> 16;
  return x;
}

__constant__ float c_mean[3] = {0.485f, 0.456f, 0.406f};
__constant__ float c_istd[3] = {1.f / 0.229f, 1.f / 0.224f, 1.f / 0.225f};

// keys[b] = hash32(id*2654435761 + salt) computed on host-agnostic 32-bit math; labels[b] likewise
__global__ void synth_labels_kernel(const long long* __restrict__ ids, int B, uint32_t salt,
                                    int num_classes, uint32_t* __restrict__ keys,
                                    long long* __restrict__ labels) {
  const int b = blockIdx.x * blockDim.x + threadIdx.x;
  if (b >= B) return;
  const uint32_t id = (uint32_t)ids[b];
  const uint32_t key = hash32(id * 2654435761u + salt);
  keys[b] = key;
  labels[b] = hash32(key ^ 0x5BD1E995u) % (uint32_t)num_classes;
}

// out: [B][S][S][8] 16-bit; pixel (c,y,x) of sample b: u = hash32(key ^ (pos * 0x27D4EB2F)) >> 8
__global__ __launch_bounds__(NT) void synth_nhwc8_kernel(const uint32_t* __restrict__ keys,
                                                         const long long* __restrict__ labels,
                                                         int B, int S, void* __restrict__ out, int dt) {
  const long long npix = (long long)B * S * S;
  const int hw = S * S;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < npix; i += (long long)gridDim.x * NT) {
    const int b = (int)(i / hw);
    const int pix = (int)(i - (long long)b * hw);
    const uint32_t key = keys[b];
    const long long lab = labels[b];
    float h[8];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const uint32_t pos = (uint32_t)(c * hw + pix);
      const uint32_t u = hash32(key ^ (pos * 0x27D4EB2Fu)) >> 8;
      const float uf = (float)u * (1.0f / 16777216.0f);
      const float tint = (float)((lab * (2 * c + 3) + c) % 4) / 3.0f;
      const float v = (uf * 0.5f + 0.5f * tint - c_mean[c]) * c_istd[c];
      h[c] = v;
    }
#pragma unroll
    for (int c = 3; c < 8; ++c) h[c] = 0.f;
#pragma unroll
    for (int c = 0; c < 8; ++c) st_any(out, (size_t)i * 8 + c, h[c], dt);
  }
}

__global__ __launch_bounds__(NT) void nchw_to_nhwc8_kernel(const float* __restrict__ x, int B, int C,
                                                           int H, int W, void* __restrict__ out,
                                                           int dt) {
  const long long npix = (long long)B * H * W;
  const int hw = H * W;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < npix; i += (long long)gridDim.x * NT) {
    const int b = (int)(i / hw);
    const int pix = (int)(i - (long long)b * hw);
#pragma unroll
    for (int c = 0; c < 8; ++c) {
      const float v = c < C ? x[((size_t)b * C + c) * hw + pix] : 0.f;
      st_any(out, (size_t)i * 8 + c, v, dt);
    }
  }
}

// ------------------------------------------------------------------ stem space-to-depth
// The 7x7/2 stem on a 3-channel image is re-expressed as a 4x4/1 conv (pad 2, output S/2) on the
// 2x2 space-to-depth image X'[i][j][(p*2+q)*3+c] = x[2i+p][2j+q][c] (12 channels padded to 16):
// y[o] = sum_{a,b in -2..1} X'[o+a] . W'[a+2][b+2], W'[a+2][b+2][(p,q,c)] = w[2a+p+3][2b+q+3][c].
// K = 16 taps x 16 channels = 256: whole 16-B chunks, MFMA-aligned, no per-chunk tap decode.
__global__ __launch_bounds__(NT) void synth_s2d_kernel(const uint32_t* __restrict__ keys,
                                                       const long long* __restrict__ labels,
                                                       int B, int S, void* __restrict__ out, int dt) {
  const int S2 = S / 2;
  const long long npix = (long long)B * S2 * S2;
  const int hw = S * S;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < npix; i += (long long)gridDim.x * NT) {
    const int b = (int)(i / (S2 * S2));
    const int rem = (int)(i - (long long)b * S2 * S2);
    const int oi = rem / S2, oj = rem - oi * S2;
    const uint32_t key = keys[b];
    const long long lab = labels[b];
    float h[16];
#pragma unroll
    for (int pq = 0; pq < 4; ++pq) {
      const int pix = (2 * oi + (pq >> 1)) * S + 2 * oj + (pq & 1);
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const uint32_t pos = (uint32_t)(c * hw + pix);
        const uint32_t u = hash32(key ^ (pos * 0x27D4EB2Fu)) >> 8;
        const float uf = (float)u * (1.0f / 16777216.0f);
        const float tint = (float)((lab * (2 * c + 3) + c) % 4) / 3.0f;
        const float v = (uf * 0.5f + 0.5f * tint - c_mean[c]) * c_istd[c];
        h[pq * 3 + c] = v;
      }
    }
#pragma unroll
    for (int c = 12; c < 16; ++c) h[c] = 0.f;
    if (dt == DT_F32) {
      store8<DT_F32>(out, (size_t)i * 16, h);
      store8<DT_F32>(out, (size_t)i * 16 + 8, h + 8);
    } else if (dt == DT_BF16) {
      store8<DT_BF16>(out, (size_t)i * 16, h);
      store8<DT_BF16>(out, (size_t)i * 16 + 8, h + 8);
    } else {
      store8<DT_F16>(out, (size_t)i * 16, h);
      store8<DT_F16>(out, (size_t)i * 16 + 8, h + 8);
    }
  }
}

__global__ __launch_bounds__(NT) void nchw_to_s2d_kernel(const float* __restrict__ x, int B, int C,
                                                         int S, void* __restrict__ out, int dt) {
  const int S2 = S / 2;
  const long long npix = (long long)B * S2 * S2;
  for (long long i = blockIdx.x * (long long)NT + threadIdx.x; i < npix; i += (long long)gridDim.x * NT) {
    const int b = (int)(i / (S2 * S2));
    const int rem = (int)(i - (long long)b * S2 * S2);
    const int oi = rem / S2, oj = rem - oi * S2;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int pq = k / 3, c = k - pq * 3;
      float v = 0.f;
      if (k < 12 && c < C)
        v = x[(((size_t)b * C + c) * S + 2 * oi + (pq >> 1)) * S + 2 * oj + (pq & 1)];
      st_any(out, (size_t)i * 16 + k, v, dt);
    }
  }
}

// src f32 OHWI [64][7][7][3] -> dst 16-bit [64][4][4][16]
__global__ void pack_stem_s2d_kernel(const float* __restrict__ src, void* __restrict__ dst, int Cout,
                                     int dt) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Cout * 256) return;
  const int co = i >> 8, k = i & 255;
  const int tap = k >> 4, ch = k & 15;
  const int ra = tap >> 2, sb = tap & 3;
  float v = 0.f;
  if (ch < 12) {
    const int pq = ch / 3, c = ch - pq * 3;
    const int r = 2 * ra + (pq >> 1) - 1, s = 2 * sb + (pq & 1) - 1;
    if (r >= 0 && r < 7 && s >= 0 && s < 7) v = src[(((size_t)co * 7 + r) * 7 + s) * 3 + c];
  }
  st_any(dst, i, v, dt);
}

// gradient of the packed weight [64][256] (f32) -> OHWI [64][7][7][3] of the master weight
__global__ void stem_s2d_grad_kernel(const float* __restrict__ gp, float* __restrict__ g, int Cout,
                                     int accumulate) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Cout * 147) return;
  const int co = i / 147, rem = i - co * 147;
  const int r = rem / 21, s = (rem / 3) % 7, c = rem % 3;
  const int p = (r + 1) & 1, q = (s + 1) & 1;
  const int ra = (r + 1 - p) >> 1, sb = (s + 1 - q) >> 1;
  const float v = gp[(size_t)co * 256 + (ra * 4 + sb) * 16 + (p * 2 + q) * 3 + c];
  g[i] = accumulate ? g[i] + v : v;
}

inline int grid_for(long long n, int cap = 4096) {
  long long b = (n + NT - 1) / NT;
  return (int)(b < 1 ? 1 : (b > cap ? cap : b));
}

}  // namespace

// Streaming probe for tools/fork_bench.py: dst = 2 * src over n floats; launched through
// hipExtLaunchKernelGGL when ``stop`` is given, so the kernel dispatch itself completes that event
// (no separate marker on the stream) -- the cheapest fork point a second stream can wait on.
__global__ __launch_bounds__(256) void fork_probe_kernel(float* __restrict__ dst,
                                                         const float* __restrict__ src, int n) {
  for (int i = (blockIdx.x * 256 + threadIdx.x) * 4; i < n; i += gridDim.x * 256 * 4)
    *reinterpret_cast<f32x4*>(dst + i) = 2.f * *reinterpret_cast<const f32x4*>(src + i);
}

thread_local hipStream_t g_trk_stream = nullptr;
thread_local hipEvent_t g_trk_event = nullptr;
thread_local unsigned long long g_trk_count = 0;

extern "C" {

// Arm (ev != null) / disarm fork tracking of this host thread's launches on stream st (common.h).
int pda_track(hipStream_t st, hipEvent_t ev) {
  g_trk_stream = st;
  g_trk_event = ev;
  return 0;
}
unsigned long long pda_track_count() { return g_trk_count; }
int pda_event_create(hipEvent_t* ev) { return (int)hipEventCreateWithFlags(ev, hipEventDisableTiming); }
// flags: hipEventDisableTiming | optionally hipEventDisableSystemFence (the fork events are only
// waited on by a stream of the same device: an agent-scope release is enough)
int pda_event_create_flags(hipEvent_t* ev, unsigned flags) { return (int)hipEventCreateWithFlags(ev, flags); }
int pda_event_record(hipEvent_t ev, hipStream_t st) { return (int)hipEventRecord(ev, st); }
int pda_event_destroy(hipEvent_t ev) { return (int)hipEventDestroy(ev); }
int pda_stream_wait_event(hipStream_t st, hipEvent_t ev) { return (int)hipStreamWaitEvent(st, ev, 0); }

int pda_fork_probe(float* dst, const float* src, int n, hipEvent_t stop, hipStream_t st) {
  if (n % 4) return -2;
  const dim3 grid(2048), block(256);
  if (stop != nullptr)
    hipExtLaunchKernelGGL(fork_probe_kernel, grid, block, 0, st, nullptr, stop, 0, dst, src, n);
  else
    TRACKED_LAUNCH(fork_probe_kernel, grid, block, 0, st, dst, src, n);
  return (int)hipGetLastError();
}

int pda_xent(const float* logits, int B, int K, int ld_in, const long long* labels, float* loss_rows,
             float* loss, void* dlog, int ld_out, float gscale, const float* gdev, int dt,
             int want_grad, hipStream_t st) {
  TRACKED_LAUNCH(xent_kernel, dim3((B + 3) / 4), dim3(NT), 0, st, logits, B, K, ld_in, labels,
                     loss_rows, dlog, ld_out, gscale, gdev, dt, want_grad);
  if (loss) TRACKED_LAUNCH(mean_kernel, dim3(1), dim3(1024), 0, st, loss_rows, B, loss);
  return (int)hipGetLastError();
}

int pda_topk(const float* logits, int B, int K, int ld, const long long* labels, float* hits,
             hipStream_t st) {
  TRACKED_LAUNCH(topk_kernel, dim3((B + 3) / 4), dim3(NT), 0, st, logits, B, K, ld, labels, hits);
  return (int)hipGetLastError();
}

int pda_col_sum(const void* x, int rows, int C, int ld, float scale, float* out, int dt,
                int accumulate, hipStream_t st) {
  TRACKED_LAUNCH(col_sum_kernel, dim3((C + 63) / 64), dim3(1024), 0, st, x, rows, C, ld,
                     scale, out, dt, accumulate);
  return (int)hipGetLastError();
}

int pda_sgd_flat(float* p, float* g, float* buf, void* shadow, long long n, float lr, float momentum,
                 float wd, const float* scale, const float* found_inf, int flags, int dt,
                 hipStream_t st) {
  TRACKED_LAUNCH(sgd_flat_kernel, dim3(grid_for(n / 4 + 1, 8192)), dim3(NT), 0, st, p, g, buf,
                     (u16*)shadow, n, lr, momentum, wd, scale, found_inf, flags, dt);
  return (int)hipGetLastError();
}

int pda_cast_flat(const float* p, void* s, long long n, int dt, hipStream_t st) {
  TRACKED_LAUNCH(cast_flat_kernel, dim3(grid_for(n, 8192)), dim3(NT), 0, st, p, (u16*)s, n, dt);
  return (int)hipGetLastError();
}

int pda_amp_scan(const float* g, long long n, float* found_inf, float* inv, float* scale,
                 int* tracker, int* ws, float growth, float backoff, int interval, hipStream_t st) {
  TRACKED_LAUNCH(amp_scan_kernel, dim3(grid_for(n / 4 + 1, 2048)), dim3(NT), 0, st, g, n,
                     found_inf, inv, scale, tracker, ws, growth, backoff, interval);
  return (int)hipGetLastError();
}

int pda_pack_stem(const float* src, void* dst, int Cout, int RS, int Cin, int Cpad, int Kpad, int dt,
                  hipStream_t st) {
  const int n = Cout * Kpad;
  TRACKED_LAUNCH(pack_stem_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, dst, Cout,
                     RS, Cin, Cpad, Kpad, dt);
  return (int)hipGetLastError();
}

int pda_synth(const long long* ids, int B, unsigned salt, int num_classes, unsigned* keys,
              long long* labels, int S, void* out, int dt, hipStream_t st) {
  TRACKED_LAUNCH(synth_labels_kernel, dim3((B + 255) / 256), dim3(256), 0, st, ids, B, salt,
                     num_classes, keys, labels);
  TRACKED_LAUNCH(synth_nhwc8_kernel, dim3(grid_for((long long)B * S * S, 8192)), dim3(NT), 0, st,
                     keys, labels, B, S, out, dt);
  return (int)hipGetLastError();
}

int pda_synth_s2d(const long long* ids, int B, unsigned salt, int num_classes, unsigned* keys,
                  long long* labels, int S, void* out, int dt, hipStream_t st) {
  TRACKED_LAUNCH(synth_labels_kernel, dim3((B + 255) / 256), dim3(256), 0, st, ids, B, salt,
                     num_classes, keys, labels);
  TRACKED_LAUNCH(synth_s2d_kernel, dim3(grid_for((long long)B * (S / 2) * (S / 2), 8192)), dim3(NT),
                     0, st, keys, labels, B, S, out, dt);
  return (int)hipGetLastError();
}

int pda_nchw_to_s2d(const float* x, int B, int C, int S, void* out, int dt, hipStream_t st) {
  TRACKED_LAUNCH(nchw_to_s2d_kernel, dim3(grid_for((long long)B * (S / 2) * (S / 2), 8192)),
                     dim3(NT), 0, st, x, B, C, S, out, dt);
  return (int)hipGetLastError();
}

int pda_pack_stem_s2d(const float* src, void* dst, int Cout, int dt, hipStream_t st) {
  TRACKED_LAUNCH(pack_stem_s2d_kernel, dim3((Cout * 256 + 255) / 256), dim3(256), 0, st, src,
                     dst, Cout, dt);
  return (int)hipGetLastError();
}

int pda_stem_s2d_grad(const float* gp, float* g, int Cout, int accumulate, hipStream_t st) {
  TRACKED_LAUNCH(stem_s2d_grad_kernel, dim3((Cout * 147 + 255) / 256), dim3(256), 0, st, gp, g,
                     Cout, accumulate);
  return (int)hipGetLastError();
}

int pda_nchw_to_nhwc8(const float* x, int B, int C, int H, int W, void* out, int dt, hipStream_t st) {
  TRACKED_LAUNCH(nchw_to_nhwc8_kernel, dim3(grid_for((long long)B * H * W, 8192)), dim3(NT), 0, st,
                     x, B, C, H, W, out, dt);
  return (int)hipGetLastError();
}

}  // extern "C"
