// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of pytorch_distributed_amd.
// Wave64 everywhere; 16-bit element types are moved as raw shorts and bit-cast at the MFMA.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <stdint.h>
#include <cstdlib>

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef int i32x4 __attribute__((ext_vector_type(4)));

// LDS-DMA (buffer_load_dwordx4 ... lds): buffer descriptor (base, num_records bytes; offsets past
// it read 0) in SGPRs, and one 16-B-per-lane piece (64 lanes -> 1 KiB at lds, lane-linear; lds
// wave-uniform: it becomes M0). Written in asm: hipcc tracks the builtin's DMA as a pending LDS
// store and, in loops with transposed (ds_read_b64_tr_b16) reads, waits vmcnt(0) before the first
// such read of every step -- draining every tile the loop keeps in flight. The asm DMA is invisible
// to that bookkeeping; the kernels count their DMAs themselves (counted s_waitcnt vmcnt). M0 is
// compiler-reserved: saved and restored in the statement. s_nop 4: the descriptor may come fresh
// from a VALU (readfirstlane).
typedef int dma_rsrc_t __attribute__((ext_vector_type(4)));
__device__ __forceinline__ dma_rsrc_t dma_rsrc(const void* base, uint32_t bytes) {
  const uint64_t b = (uint64_t)(uintptr_t)base;
  return dma_rsrc_t{(int)(uint32_t)b, (int)(uint32_t)(b >> 32), (int)bytes, 0x00020000};
}
__device__ __forceinline__ void dma16_asm(dma_rsrc_t r, char* lds, uint32_t voff) {
  const uint32_t l = __builtin_amdgcn_readfirstlane(
      (uint32_t)(uintptr_t)(__attribute__((address_space(3))) char*)lds);
  uint32_t keep;
  asm volatile("s_nop 4\n\ts_mov_b32 %0, m0\n\ts_mov_b32 m0, %3\n\ts_nop 0\n\t"
               "buffer_load_dwordx4 %1, %2, 0 offen lds\n\ts_mov_b32 m0, %0"
               : "=&s"(keep) : "v"(voff), "s"(r), "s"(l) : "memory");
}
typedef unsigned short u16;

#define LDS_PTR(T, p) ((__attribute__((address_space(3))) T*)(p))

// dtype tags shared with the Python side (ops/ext.py)
// DT_F32S: f32 tensors in memory, products on the bf16 MFMA as a three-term split
// (a_hi*b_hi + a_hi*b_lo + a_lo*b_hi, hi = bf16(x), lo = bf16(x - hi)): ~16 significant bits
// per product, above the TF32 (10-bit) convolutions of the reference's "fp32" runs
enum DType : int { DT_F32 = 0, DT_BF16 = 1, DT_F16 = 2, DT_F32S = 3 };

// ---- 16-bit <-> f32 conversions -------------------------------------------------------------
__device__ __forceinline__ float bf16_to_f32(u16 v) { return __uint_as_float(((uint32_t)v) << 16); }
__device__ __forceinline__ u16 f32_to_bf16(float f) {
  __bf16 b = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN stays NaN
  return __builtin_bit_cast(u16, b);
}
__device__ __forceinline__ float f16_to_f32(u16 v) { return (float)__builtin_bit_cast(_Float16, v); }
__device__ __forceinline__ u16 f32_to_f16(float f) { return __builtin_bit_cast(u16, (_Float16)f); }

// packed pairs: one dword = two 16-bit elements (lo = first). Conversions use the packed
// instructions (v_cvt_pk_bf16_f32 / v_cvt_pk_f16 RNE) and f32x2 math maps to v_pk_{add,mul,fma}_f32.
typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
template <int DT> __device__ __forceinline__ uint32_t pack2(f32x2 v);
template <> __device__ __forceinline__ uint32_t pack2<DT_BF16>(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2));
}
template <> __device__ __forceinline__ uint32_t pack2<DT_F16>(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, f16x2));
}
// BatchNorm-backward apply dy = k1*dz + k2*y + k3 as ONE explicit fma chain, shared by the apply
// kernels (bn.hip) and the WGRAD_BNA operand staging (conv_gemm.hip) so the two paths round alike.
__device__ __forceinline__ float bnb_affine(float k1, float k2, float k3, float dz, float y) {
  return __builtin_fmaf(k1, dz, __builtin_fmaf(k2, y, k3));
}
__device__ __forceinline__ f32x2 bnb_affine2(f32x2 k1, f32x2 k2, f32x2 k3, f32x2 dz, f32x2 y) {
  return f32x2{bnb_affine(k1.x, k2.x, k3.x, dz.x, y.x), bnb_affine(k1.y, k2.y, k3.y, dz.y, y.y)};
}
// BatchNorm apply of a residual block's tail, before the ReLU: bn(y) [+ r (mode 1) | + bn2(r)
// (mode 2)], as explicit fmas shared by the apply kernels (bn.hip) and the FWD_TAIL conv prologue
// (conv_gemm.hip), so the activation one of them writes is bit-identical to the other's.
__device__ __forceinline__ f32x2 tail_pre2(f32x2 y, f32x2 a, f32x2 b, f32x2 r, f32x2 a2, f32x2 b2,
                                           int mode) {
  f32x2 v = f32x2{__builtin_fmaf(y.x, a.x, b.x), __builtin_fmaf(y.y, a.y, b.y)};
  if (mode) {
    if (mode == 2) r = f32x2{__builtin_fmaf(r.x, a2.x, b2.x), __builtin_fmaf(r.y, a2.y, b2.y)};
    v = f32x2{v.x + r.x, v.y + r.y};
  }
  return v;
}
template <int DT> __device__ __forceinline__ f32x2 unpack2(uint32_t w);
template <> __device__ __forceinline__ f32x2 unpack2<DT_BF16>(uint32_t w) {
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
template <> __device__ __forceinline__ f32x2 unpack2<DT_F16>(uint32_t w) {
  return __builtin_convertvector(__builtin_bit_cast(f16x2, w), f32x2);
}

template <int DT> __device__ __forceinline__ float ld16(u16 v);
template <> __device__ __forceinline__ float ld16<DT_BF16>(u16 v) { return bf16_to_f32(v); }
template <> __device__ __forceinline__ float ld16<DT_F16>(u16 v) { return f16_to_f32(v); }
template <int DT> __device__ __forceinline__ u16 st16(float f);
template <> __device__ __forceinline__ u16 st16<DT_BF16>(float f) { return f32_to_bf16(f); }
template <> __device__ __forceinline__ u16 st16<DT_F16>(float f) { return f32_to_f16(f); }

// ---- MFMA 16x16x32 (bf16 / f16 inputs, f32 accumulate) --------------------------------------
template <int DT> __device__ __forceinline__ f32x4 mfma16(s16x8 a, s16x8 b, f32x4 c);
template <> __device__ __forceinline__ f32x4 mfma16<DT_BF16>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), c, 0, 0, 0);
}
template <> __device__ __forceinline__ f32x4 mfma16<DT_F16>(s16x8 a, s16x8 b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8, a),
                                                __builtin_bit_cast(f16x8, b), c, 0, 0, 0);
}

// ---- MFMA 16x16x4 f32 (exact fp32 path, MX_DTYPE=fp32) --------------------------------------
__device__ __forceinline__ f32x4 mfma16_f32(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ---- 8 consecutive activation elements of any storage dtype <-> f32[8] -------------------------
// 16-bit: one 16-B chunk; f32: two. Element offsets (not bytes) index the tensor.
template <int DT> struct Raw8 { i32x4 v; };
template <> struct Raw8<DT_F32> { f32x4 a, b; };

template <int DT> __device__ __forceinline__ Raw8<DT> ldraw8(const void* base, size_t idx) {
  Raw8<DT> r;
  if constexpr (DT == DT_F32) {
    const f32x4* p = reinterpret_cast<const f32x4*>(reinterpret_cast<const float*>(base) + idx);
    r.a = p[0];
    r.b = p[1];
  } else {
    r.v = *reinterpret_cast<const i32x4*>(reinterpret_cast<const u16*>(base) + idx);
  }
  return r;
}
template <int DT> __device__ __forceinline__ void straw8(void* base, size_t idx, const Raw8<DT>& r) {
  if constexpr (DT == DT_F32) {
    f32x4* p = reinterpret_cast<f32x4*>(reinterpret_cast<float*>(base) + idx);
    p[0] = r.a;
    p[1] = r.b;
  } else {
    *reinterpret_cast<i32x4*>(reinterpret_cast<u16*>(base) + idx) = r.v;
  }
}
template <int DT> __device__ __forceinline__ void cvt8(const Raw8<DT>& r, float* f) {
  if constexpr (DT == DT_F32) {
#pragma unroll
    for (int e = 0; e < 4; ++e) { f[e] = r.a[e]; f[4 + e] = r.b[e]; }
  } else {
    const u16* h = reinterpret_cast<const u16*>(&r.v);
#pragma unroll
    for (int e = 0; e < 8; ++e) f[e] = DT == DT_BF16 ? bf16_to_f32(h[e]) : f16_to_f32(h[e]);
  }
}
template <int DT> __device__ __forceinline__ Raw8<DT> pk8(const float* f) {
  Raw8<DT> r;
  if constexpr (DT == DT_F32) {
#pragma unroll
    for (int e = 0; e < 4; ++e) { r.a[e] = f[e]; r.b[e] = f[4 + e]; }
  } else {
    u16* h = reinterpret_cast<u16*>(&r.v);
#pragma unroll
    for (int e = 0; e < 8; ++e) h[e] = DT == DT_BF16 ? f32_to_bf16(f[e]) : f32_to_f16(f[e]);
  }
  return r;
}
template <int DT> __device__ __forceinline__ void load8(const void* base, size_t idx, float* f) {
  cvt8<DT>(ldraw8<DT>(base, idx), f);
}
template <int DT> __device__ __forceinline__ void store8(void* base, size_t idx, const float* f) {
  straw8<DT>(base, idx, pk8<DT>(f));
}

// runtime-dtype scalar access (small kernels: data generation, head, optimizer shadow)
__device__ __forceinline__ void st_any(void* base, size_t i, float v, int dt) {
  if (dt == DT_F32) reinterpret_cast<float*>(base)[i] = v;
  else reinterpret_cast<u16*>(base)[i] = dt == DT_BF16 ? f32_to_bf16(v) : f32_to_f16(v);
}
__device__ __forceinline__ float ld_any(const void* base, size_t i, int dt) {
  if (dt == DT_F32) return reinterpret_cast<const float*>(base)[i];
  const u16 h = reinterpret_cast<const u16*>(base)[i];
  return dt == DT_BF16 ? bf16_to_f32(h) : f16_to_f32(h);
}

// ---- fast unsigned division by a runtime constant (n < 2^31) --------------------------------
struct FastDiv {
  uint32_t d, m, s;
};
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
  return (__umulhi(n, f.m) + n) >> f.s;
}

// ---- wave / block reductions ---------------------------------------------------------------
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// XCD-aware bijective remap of a 1-D block index: consecutive *logical* tiles land on the same
// XCD (blocks b and b+8 share an XCD under round-robin dispatch), so neighbouring tiles that share
// an operand panel hit the same L2. Speed only -- never correctness (cdna_hip_programming.md T1).
__device__ __forceinline__ uint32_t xcd_remap(uint32_t bid, uint32_t nwg) {
  const uint32_t q = nwg >> 3, r = nwg & 7, x = bid & 7;
  const uint32_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  return base + (bid >> 3);
}
// Launches that walk their tiles / items from the end (xcd_remap_rev, the stem pool's reversed
// grid-stride loop): PDA_REVERSE lists them ("fwd_tail", "bnf", "stem_pool"; "none": none); default
// all three -- their producers (conv3, the tail-epilogue data gradient, the stem conv) ran just
// before and wrote those tiles last, so up to 256 MiB of their reads hit the Infinity Cache
// (profiles/ab_r6.md section 13: -0.08 ms/step)
inline const char* pda_reverse_env() {
  const char* e = getenv("PDA_REVERSE");
  return e ? e : "fwd_tail+bnf+stem_pool";
}
// the same XCD chunks, each walked from its end: a consumer launched right after a producer of the
// same chunking reads first what the producer wrote last (still in the 256 MiB Infinity Cache)
__device__ __forceinline__ uint32_t xcd_remap_rev(uint32_t bid, uint32_t nwg) {
  const uint32_t q = nwg >> 3, r = nwg & 7, x = bid & 7;
  const uint32_t base = x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q;
  const uint32_t len = x < r ? q + 1 : q;
  return base + (len - 1 - (bid >> 3));
}

// ---------------------------------------------------------------------------------------------
// Fork tracking (models/native.py _fork_side, csrc/misc.hip pda_track): while armed for this host
// thread, every launch on the tracked stream completes g_trk_event through its own dispatch
// (hipExtLaunchKernel stop event), so a second stream can wait for "the latest launch on the main
// stream" without an event-record marker between kernels (~4-5 us of main-stream bubble per fork
// measured by tools/fork_bench.py; the stop event costs ~nothing when nobody waits).
extern thread_local hipStream_t g_trk_stream;
extern thread_local hipEvent_t g_trk_event;
extern thread_local unsigned long long g_trk_count;   // tracked launches so far (this thread)
#define TRACKED_LAUNCH(K, G, B, S, ST, ...)                                                        \
  do {                                                                                         \
    hipStream_t pda_st_ = (ST);                                                                \
    if (g_trk_event != nullptr && pda_st_ == g_trk_stream) {                                   \
      hipExtLaunchKernelGGL(K, G, B, S, pda_st_, nullptr, g_trk_event, 0, __VA_ARGS__);        \
      ++g_trk_count;                                                                           \
    } else                                                                                     \
      hipLaunchKernelGGL(K, G, B, S, pda_st_, __VA_ARGS__);                                    \
  } while (0)
