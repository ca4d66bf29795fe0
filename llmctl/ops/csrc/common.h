// Shared helpers for llmctl's CDNA4 (gfx950) HIP kernels.
//
// Conventions
//   * wave64: every warp-level idiom here is written for 64 lanes (shfl_xor offsets up to 32).
//   * bf16 tensors are moved as 16-byte vectors (8 x bf16 per lane) — hipcc does not
//     auto-vectorise bf16 (CDNA guide, Guideline 13).
//   * f32 -> bf16 uses the compiler's RNE cast (lowers to v_cvt_pk_bf16_f32, NaN-safe).
#pragma once

#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <ATen/ATen.h>
#include <ATen/hip/HIPContext.h>
#include <c10/core/DeviceGuard.h>
#include <ATen/hip/impl/HIPStreamMasqueradingAsCUDA.h>
#include <torch/library.h>

#include <cstdint>

#define LLMCTL_CHECK(cond, ...) TORCH_CHECK(cond, "llmctl: ", __VA_ARGS__)
#define LLMCTL_CHECK_CUDA(t) LLMCTL_CHECK((t).is_cuda(), #t " must be a GPU tensor")
#define LLMCTL_CHECK_CONTIG(t) LLMCTL_CHECK((t).is_contiguous(), #t " must be contiguous")
#define LLMCTL_CHECK_BF16(t) LLMCTL_CHECK((t).scalar_type() == at::kBFloat16, #t " must be bf16")
#define LLMCTL_HIP_CHECK(expr)                                                      \
  do {                                                                              \
    hipError_t _e = (expr);                                                         \
    TORCH_CHECK(_e == hipSuccess, "llmctl HIP error: ", hipGetErrorString(_e));     \
  } while (0)

namespace llmctl {

// llmctl.config.knobs (knobs.cpp): value pushed from Python, else the default
int64_t knob(const char* name, int64_t dflt);

using bf16x8 = __attribute__((ext_vector_type(8))) unsigned short;  // 16 B
using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ float bf2f(unsigned short u) { return __uint_as_float(((unsigned)u) << 16); }

__device__ __forceinline__ unsigned short f2bf(float f) {
  __hip_bfloat16 b = __float2bfloat16(f);
  return __bfloat16_as_ushort(b);
}

__device__ __forceinline__ void load8(const unsigned short* p, float* out) {
  bf16x8 v = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) out[j] = bf2f(v[j]);
}

__device__ __forceinline__ void store8(unsigned short* p, const float* in) {
  bf16x8 v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = f2bf(in[j]);
  *reinterpret_cast<bf16x8*>(p) = v;
}

// ---- paged KV cache element: bf16, or OCP fp8 e4m3fn (gfx950's v_cvt_pk_*fp8*; saturating at
//      +-448, scale 1: torch.float8_e4m3fn bit patterns).  A row of 8 elements is 16 B / 8 B.
__device__ __forceinline__ float sat_fp8(float x) { return __builtin_amdgcn_fmed3f(x, -448.f, 448.f); }

__device__ __forceinline__ uint2 f32x8_to_fp8(const float* x) {
  int lo = 0, hi = 0;
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(sat_fp8(x[0]), sat_fp8(x[1]), lo, false);
  lo = __builtin_amdgcn_cvt_pk_fp8_f32(sat_fp8(x[2]), sat_fp8(x[3]), lo, true);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(sat_fp8(x[4]), sat_fp8(x[5]), hi, false);
  hi = __builtin_amdgcn_cvt_pk_fp8_f32(sat_fp8(x[6]), sat_fp8(x[7]), hi, true);
  return make_uint2((unsigned)lo, (unsigned)hi);
}

__device__ __forceinline__ void fp8x8_to_f32(uint2 u, float* out) {
  const auto a = __builtin_amdgcn_cvt_pk_f32_fp8((int)u.x, false), b = __builtin_amdgcn_cvt_pk_f32_fp8((int)u.x, true);
  const auto c = __builtin_amdgcn_cvt_pk_f32_fp8((int)u.y, false), d = __builtin_amdgcn_cvt_pk_f32_fp8((int)u.y, true);
  out[0] = a[0], out[1] = a[1], out[2] = b[0], out[3] = b[1];
  out[4] = c[0], out[5] = c[1], out[6] = d[0], out[7] = d[1];
}

// 8 cache elements starting at element index e of a cache of either type
__device__ __forceinline__ void cache_store8(void* base, long e, const float* x, bool fp8) {
  if (fp8) *reinterpret_cast<uint2*>(static_cast<unsigned char*>(base) + e) = f32x8_to_fp8(x);
  else store8(static_cast<unsigned short*>(base) + e, x);
}
__device__ __forceinline__ void cache_load8(const void* base, long e, float* x, bool fp8) {
  if (fp8) fp8x8_to_f32(*reinterpret_cast<const uint2*>(static_cast<const unsigned char*>(base) + e), x);
  else load8(static_cast<const unsigned short*>(base) + e, x);
}
// ... as 8 bf16 (16 B) for an LDS image.  An e4m3 value (3 mantissa bits) is exact in bf16, so its
// f32 image has a zero low half: the bf16 is the f32's high 16 bits (one v_perm_b32 per pair).
__device__ __forceinline__ uint4 cache_load8_bf16(const void* base, long e, bool fp8) {
  if (!fp8) return *reinterpret_cast<const uint4*>(static_cast<const unsigned short*>(base) + e);
  float x[8];
  fp8x8_to_f32(*reinterpret_cast<const uint2*>(static_cast<const unsigned char*>(base) + e), x);
  unsigned w[4];
#pragma unroll
  for (int j = 0; j < 4; ++j)
    w[j] = __builtin_amdgcn_perm(__float_as_uint(x[2 * j + 1]), __float_as_uint(x[2 * j]), 0x07060302u);
  return make_uint4(w[0], w[1], w[2], w[3]);
}

// host: a paged KV cache tensor is bf16 or fp8 e4m3fn
inline bool kv_fp8(const at::Tensor& c) { return c.scalar_type() == at::kFloat8_e4m3fn; }
inline bool kv_cache_ok(const at::Tensor& c) { return c.scalar_type() == at::kBFloat16 || kv_fp8(c); }

// Workgroup barrier ordering LDS only: __syncthreads() is also a release for global memory
// (s_waitcnt vmcnt(0)), which would drain in-flight prefetch loads and no-return atomics
// (~3k cycles each under load) at every barrier.  LDS-scoped fences lower to lgkmcnt(0).
__device__ __forceinline__ void lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}

// block-wide sum for blockDim.x = NW*64 (result valid in every thread)
template <int NW>
__device__ __forceinline__ float block_sum(float v, float* smem) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  if (l == 0) smem[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) r += smem[i];
  __syncthreads();
  return r;
}

// torch on ROCm "masquerades" HIP as the CUDA device type: use the masquerading stream so
// kernels honour torch.cuda.stream(...) contexts and hipGraph capture.
inline hipStream_t stream() { return at::hip::getCurrentHIPStreamMasqueradingAsCUDA().stream(); }

inline int num_cus() {
  static int n = -1;
  if (n < 0) {
    hipDeviceProp_t p;
    int dev = 0;
    LLMCTL_HIP_CHECK(hipGetDevice(&dev));
    LLMCTL_HIP_CHECK(hipGetDeviceProperties(&p, dev));
    n = p.multiProcessorCount;
  }
  return n;
}

template <typename T>
inline const unsigned short* bf_ptr(const T& t) {
  return reinterpret_cast<const unsigned short*>(t.data_ptr());
}
template <typename T>
inline unsigned short* bf_mut(T& t) {
  return reinterpret_cast<unsigned short*>(t.data_ptr());
}

}  // namespace llmctl
