// Memory-bound elementwise kernels (gfx950): RoPE fused with the QKV split, SwiGLU, GELU.
//
// All bf16 traffic is 16-byte vectors; RoPE reads host-precomputed fp32 cos/sin tables
// (CDNA guide App. B: on-device sin/cos turns RoPE VALU-bound).  RoPE uses the rotate-half
// (NeoX/Llama) convention; the backward is the transposed rotation and writes straight
// into the [T, (nq+2nkv)*D] gradient of the QKV GEMM output, so no concat/copy is needed.
#include "common.h"

namespace llmctl {
namespace {

template <typename PosT>
__global__ __launch_bounds__(256) void rope_fwd_kernel(const unsigned short* __restrict__ qkv,
                                                        const float* __restrict__ cosT,
                                                        const float* __restrict__ sinT,
                                                        const PosT* __restrict__ pos, unsigned short* __restrict__ q,
                                                        unsigned short* __restrict__ k,
                                                        unsigned short* __restrict__ v, int nq, int nkv, int D,
                                                        int S, long total, void* __restrict__ kc = nullptr,
                                                        void* __restrict__ vc = nullptr,
                                                        const int64_t* __restrict__ slots = nullptr, bool kv8 = false) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int CH = D >> 4;
  const int NH = nq + 2 * nkv;
  const int c = idx % CH;
  const long r = idx / CH;
  const int h = r % NH;
  const long t = r / NH;
  const int half = D >> 1;
  const unsigned short* src = qkv + (t * NH + h) * (long)D;
  float a[8], b[8], o1[8], o2[8];
  load8(src + c * 8, a);
  load8(src + half + c * 8, b);
  unsigned short* dst;
  if (h < nq + nkv) {
    const long p = pos ? (long)pos[t] : (t % S);
    const float4* cp = reinterpret_cast<const float4*>(cosT + p * half + c * 8);
    const float4* sp = reinterpret_cast<const float4*>(sinT + p * half + c * 8);
    float cs[8], sn[8];
    *reinterpret_cast<float4*>(cs) = cp[0];
    *reinterpret_cast<float4*>(cs + 4) = cp[1];
    *reinterpret_cast<float4*>(sn) = sp[0];
    *reinterpret_cast<float4*>(sn + 4) = sp[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j] * cs[j] - b[j] * sn[j];
      o2[j] = b[j] * cs[j] + a[j] * sn[j];
    }
    dst = h < nq ? q + (t * nq + h) * (long)D : k + (t * nkv + (h - nq)) * (long)D;
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j];
      o2[j] = b[j];
    }
    dst = v + (t * nkv + (h - nq - nkv)) * (long)D;
  }
  store8(dst + c * 8, o1);
  store8(dst + half + c * 8, o2);
  if (slots != nullptr && h >= nq) {  // serving: K/V rows also go straight into the paged cache
    const long sl = slots[t];
    if (sl >= 0) {
      const bool isk = h < nq + nkv;
      const long e = (sl * nkv + (isk ? h - nq : h - nq - nkv)) * (long)D;  // fp8 caches: same element index
      cache_store8(isk ? kc : vc, e + c * 8, o1, kv8);
      cache_store8(isk ? kc : vc, e + half + c * 8, o2, kv8);
    }
  }
}

template <typename PosT>
__global__ __launch_bounds__(256) void rope_bwd_kernel(const unsigned short* __restrict__ dq,
                                                        const unsigned short* __restrict__ dk,
                                                        const unsigned short* __restrict__ dv,
                                                        const float* __restrict__ cosT,
                                                        const float* __restrict__ sinT,
                                                        const PosT* __restrict__ pos,
                                                        unsigned short* __restrict__ dqkv, int nq, int nkv, int D,
                                                        int S, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int CH = D >> 4;
  const int NH = nq + 2 * nkv;
  const int c = idx % CH;
  const long r = idx / CH;
  const int h = r % NH;
  const long t = r / NH;
  const int half = D >> 1;
  const unsigned short* src;
  if (h < nq)
    src = dq + (t * nq + h) * (long)D;
  else if (h < nq + nkv)
    src = dk + (t * nkv + (h - nq)) * (long)D;
  else
    src = dv + (t * nkv + (h - nq - nkv)) * (long)D;
  float a[8], b[8], o1[8], o2[8];
  load8(src + c * 8, a);
  load8(src + half + c * 8, b);
  if (h < nq + nkv) {
    const long p = pos ? (long)pos[t] : (t % S);
    const float4* cp = reinterpret_cast<const float4*>(cosT + p * half + c * 8);
    const float4* sp = reinterpret_cast<const float4*>(sinT + p * half + c * 8);
    float cs[8], sn[8];
    *reinterpret_cast<float4*>(cs) = cp[0];
    *reinterpret_cast<float4*>(cs + 4) = cp[1];
    *reinterpret_cast<float4*>(sn) = sp[0];
    *reinterpret_cast<float4*>(sn + 4) = sp[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j] * cs[j] + b[j] * sn[j];
      o2[j] = b[j] * cs[j] - a[j] * sn[j];
    }
  } else {
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o1[j] = a[j];
      o2[j] = b[j];
    }
  }
  unsigned short* dst = dqkv + (t * NH + h) * (long)D;
  store8(dst + c * 8, o1);
  store8(dst + half + c * 8, o2);
}

__device__ __forceinline__ float sigmoidf_(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(256) void swiglu_fwd_kernel(const unsigned short* __restrict__ gu,
                                                          unsigned short* __restrict__ act, int F, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int F8 = F >> 3;
  const long t = idx / F8;
  const int c = (idx % F8) * 8;
  float g[8], u[8], o[8];
  load8(gu + t * 2 * (long)F + c, g);
  load8(gu + t * 2 * (long)F + F + c, u);
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = g[j] * sigmoidf_(g[j]) * u[j];
  store8(act + t * (long)F + c, o);
}

__global__ __launch_bounds__(256) void swiglu_bwd_kernel(const unsigned short* __restrict__ dact,
                                                          const unsigned short* __restrict__ gu,
                                                          unsigned short* __restrict__ dgu, int F, long total) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int F8 = F >> 3;
  const long t = idx / F8;
  const int c = (idx % F8) * 8;
  float g[8], u[8], d[8], og[8], ou[8];
  load8(gu + t * 2 * (long)F + c, g);
  load8(gu + t * 2 * (long)F + F + c, u);
  load8(dact + t * (long)F + c, d);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float sg = sigmoidf_(g[j]);
    const float silu = g[j] * sg;
    og[j] = d[j] * u[j] * (sg * (1.f + g[j] * (1.f - sg)));
    ou[j] = d[j] * silu;
  }
  store8(dgu + t * 2 * (long)F + c, og);
  store8(dgu + t * 2 * (long)F + F + c, ou);
}

constexpr float kGeluK = 0.7978845608028654f;  // sqrt(2/pi)

__global__ __launch_bounds__(256) void gelu_fwd_kernel(const unsigned short* __restrict__ x,
                                                        unsigned short* __restrict__ y, long n8) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  float a[8], o[8];
  load8(x + i * 8, a);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float z = kGeluK * (a[j] + 0.044715f * a[j] * a[j] * a[j]);
    o[j] = 0.5f * a[j] * (1.f + tanhf(z));
  }
  store8(y + i * 8, o);
}

__global__ __launch_bounds__(256) void gelu_bwd_kernel(const unsigned short* __restrict__ dy,
                                                        const unsigned short* __restrict__ x,
                                                        unsigned short* __restrict__ dx, long n8) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  float a[8], d[8], o[8];
  load8(x + i * 8, a);
  load8(dy + i * 8, d);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float x2 = a[j] * a[j];
    const float th = tanhf(kGeluK * (a[j] + 0.044715f * x2 * a[j]));
    const float dz = kGeluK * (1.f + 3.f * 0.044715f * x2);
    o[j] = d[j] * (0.5f * (1.f + th) + 0.5f * a[j] * (1.f - th * th) * dz);
  }
  store8(dx + i * 8, o);
}

// In-place RoPE of the q / k heads of a contiguous qkv [T, (nq + 2 nkv) D] (training forward): the
// attention kernels read q / k / v as strided views of qkv, so V is neither copied nor re-read
// (2/3 of rope_fwd_kernel's traffic).  Thread = 8 column pairs (c, c + D/2) of one (token, head);
// the grid walks (token, head) rows with 32-bit index math (T * NR * CH < 2^31, checked on the host).
template <typename PosT>
__global__ __launch_bounds__(256) void rope_inplace_kernel(unsigned short* __restrict__ qkv, const float* __restrict__ cosT,
                                                           const float* __restrict__ sinT, const PosT* __restrict__ pos,
                                                           int NR, int NH, int D, int S, int total) {
  const int idx = blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int CH = D >> 4, half = D >> 1;
  const int c = idx % CH;
  const int r = idx / CH;
  const int h = r % NR, t = r / NR;
  unsigned short* src = qkv + ((long)t * NH + h) * D;
  const long p = pos ? (long)pos[t] : (long)(t % S);
  float a[8], b[8], cs[8], sn[8], o1[8], o2[8];
  load8(src + c * 8, a);
  load8(src + half + c * 8, b);
  const float4* cp = reinterpret_cast<const float4*>(cosT + p * half + c * 8);
  const float4* sp = reinterpret_cast<const float4*>(sinT + p * half + c * 8);
  *reinterpret_cast<float4*>(cs) = cp[0];
  *reinterpret_cast<float4*>(cs + 4) = cp[1];
  *reinterpret_cast<float4*>(sn) = sp[0];
  *reinterpret_cast<float4*>(sn + 4) = sp[1];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o1[j] = a[j] * cs[j] - b[j] * sn[j];
    o2[j] = b[j] * cs[j] + a[j] * sn[j];
  }
  store8(src + c * 8, o1);
  store8(src + half + c * 8, o2);
}

inline unsigned blocks_for(long n) { return (unsigned)((n + 255) / 256); }

void check_rope_tables(const at::Tensor& c, const at::Tensor& s, int D) {
  LLMCTL_CHECK(c.is_cuda() && s.is_cuda() && c.scalar_type() == at::kFloat && s.scalar_type() == at::kFloat &&
                   c.is_contiguous() && s.is_contiguous() && c.dim() == 2 && c.size(1) == D / 2 &&
                   c.sizes() == s.sizes(),
               "cos/sin must be contiguous fp32 [P, D/2] GPU tables");
}

}  // namespace

static std::tuple<at::Tensor, at::Tensor, at::Tensor> rope_qkv_impl(
    const at::Tensor& qkv, const at::Tensor& cosT, const at::Tensor& sinT, int64_t nq, int64_t nkv, int64_t seq_len,
    const c10::optional<at::Tensor>& pos, at::Tensor* kc, at::Tensor* vc, const at::Tensor* slots) {
  LLMCTL_CHECK(qkv.is_cuda() && qkv.dim() == 2 && qkv.is_contiguous() && qkv.scalar_type() == at::kBFloat16,
               "qkv must be a contiguous 2-D bf16 GPU tensor");
  const long T = qkv.size(0);
  const int NH = nq + 2 * nkv;
  LLMCTL_CHECK(qkv.size(1) % NH == 0, "qkv width not divisible by heads");
  const int D = qkv.size(1) / NH;
  LLMCTL_CHECK(D % 16 == 0, "head_dim must be a multiple of 16");
  check_rope_tables(cosT, sinT, D);
  const bool has_pos = pos.has_value() && pos->defined() && pos->numel() > 0;
  if (has_pos) {
    LLMCTL_CHECK(pos->numel() == T && pos->is_cuda(), "positions must be [T] on GPU");
  } else {
    LLMCTL_CHECK(cosT.size(0) >= seq_len, "rope table shorter than seq_len");
  }
  const c10::DeviceGuard g(qkv.device());
  auto q = at::empty({T, nq, D}, qkv.options());
  auto k = at::empty({T, nkv, D}, qkv.options());
  auto v = at::empty({T, nkv, D}, qkv.options());
  const long total = T * NH * (D / 16);
  if (total == 0) return {q, k, v};
  void *kcp = nullptr, *vcp = nullptr;
  const int64_t* sp = nullptr;
  bool kv8 = false;
  if (slots != nullptr) {
    LLMCTL_CHECK(kc->is_contiguous() && vc->is_contiguous() && kv_cache_ok(*kc) &&
                     vc->scalar_type() == kc->scalar_type() && vc->sizes() == kc->sizes() && kc->dim() == 4 &&
                     kc->size(2) == nkv && kc->size(3) == D,
                 "k/v cache: contiguous bf16 or fp8 (e4m3fn) [blocks, block_size, Hkv, D]");
    LLMCTL_CHECK(slots->scalar_type() == at::kLong && slots->numel() == T && slots->is_contiguous(), "slots: int64 [T]");
    kcp = kc->data_ptr();
    vcp = vc->data_ptr();
    sp = slots->data_ptr<int64_t>();
    kv8 = kv_fp8(*kc);
  }
  if (has_pos && pos->scalar_type() == at::kLong)
    hipLaunchKernelGGL(rope_fwd_kernel<int64_t>, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_ptr(qkv),
                       cosT.data_ptr<float>(), sinT.data_ptr<float>(), pos->data_ptr<int64_t>(), bf_mut(q), bf_mut(k),
                       bf_mut(v), (int)nq, (int)nkv, D, (int)seq_len, total, kcp, vcp, sp, kv8);
  else
    hipLaunchKernelGGL(rope_fwd_kernel<int32_t>, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_ptr(qkv),
                       cosT.data_ptr<float>(), sinT.data_ptr<float>(),
                       has_pos ? pos->data_ptr<int32_t>() : nullptr, bf_mut(q), bf_mut(k), bf_mut(v), (int)nq,
                       (int)nkv, D, (int)seq_len, total, kcp, vcp, sp, kv8);
  return {q, k, v};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> rope_qkv_fwd(const at::Tensor& qkv, const at::Tensor& cosT,
                                                             const at::Tensor& sinT, int64_t nq, int64_t nkv,
                                                             int64_t seq_len, const c10::optional<at::Tensor>& pos) {
  return rope_qkv_impl(qkv, cosT, sinT, nq, nkv, seq_len, pos, nullptr, nullptr, nullptr);
}

// qkv [T, (nq + 2 nkv) D]: rotate the q / k heads in place (v untouched)
void rope_qk_inplace_(at::Tensor& qkv, const at::Tensor& cosT, const at::Tensor& sinT, int64_t nq, int64_t nkv,
                      int64_t seq_len, const c10::optional<at::Tensor>& pos) {
  LLMCTL_CHECK(qkv.is_cuda() && qkv.dim() == 2 && qkv.is_contiguous() && qkv.scalar_type() == at::kBFloat16,
               "rope_qk_inplace_: qkv must be a contiguous 2-D bf16 GPU tensor");
  const long T = qkv.size(0);
  const int NH = nq + 2 * nkv, NR = nq + nkv;
  LLMCTL_CHECK(qkv.size(1) % NH == 0, "qkv width not divisible by heads");
  const int D = qkv.size(1) / NH;
  LLMCTL_CHECK(D % 16 == 0, "head_dim must be a multiple of 16");
  check_rope_tables(cosT, sinT, D);
  const bool has_pos = pos.has_value() && pos->defined() && pos->numel() > 0;
  if (has_pos) {
    LLMCTL_CHECK(pos->numel() == T && pos->is_cuda() && pos->is_contiguous(), "positions must be contiguous [T] on GPU");
  } else {
    LLMCTL_CHECK(seq_len > 0 && cosT.size(0) >= seq_len, "rope table shorter than seq_len");
  }
  const long total = T * NR * (D / 16);
  LLMCTL_CHECK(total < (1L << 31), "rope_qk_inplace_: too many rows for 32-bit indexing");
  if (total == 0) return;
  const c10::DeviceGuard g(qkv.device());
  if (has_pos && pos->scalar_type() == at::kLong)
    hipLaunchKernelGGL(rope_inplace_kernel<int64_t>, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_mut(qkv),
                       cosT.data_ptr<float>(), sinT.data_ptr<float>(), pos->data_ptr<int64_t>(), NR, NH, D,
                       (int)seq_len, (int)total);
  else
    hipLaunchKernelGGL(rope_inplace_kernel<int32_t>, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_mut(qkv),
                       cosT.data_ptr<float>(), sinT.data_ptr<float>(), has_pos ? pos->data_ptr<int32_t>() : nullptr,
                       NR, NH, D, (int)std::max<int64_t>(seq_len, 1), (int)total);
}

// Serving: RoPE + split + paged-KV write in one pass (the separate kv_cache_write re-read K/V).
std::tuple<at::Tensor, at::Tensor, at::Tensor> rope_qkv_cache_fwd(const at::Tensor& qkv, const at::Tensor& cosT,
                                                                   const at::Tensor& sinT, int64_t nq, int64_t nkv,
                                                                   int64_t seq_len,
                                                                   const c10::optional<at::Tensor>& pos,
                                                                   at::Tensor& k_cache, at::Tensor& v_cache,
                                                                   const at::Tensor& slots) {
  return rope_qkv_impl(qkv, cosT, sinT, nq, nkv, seq_len, pos, &k_cache, &v_cache, &slots);
}

at::Tensor rope_qkv_bwd(const at::Tensor& dq, const at::Tensor& dk, const at::Tensor& dv, const at::Tensor& cosT,
                        const at::Tensor& sinT, int64_t seq_len, const c10::optional<at::Tensor>& pos) {
  LLMCTL_CHECK(dq.is_contiguous() && dk.is_contiguous() && dv.is_contiguous(), "grads must be contiguous");
  const long T = dq.size(0);
  const int nq = dq.size(1), nkv = dk.size(1), D = dq.size(2);
  check_rope_tables(cosT, sinT, D);
  const bool has_pos = pos.has_value() && pos->defined() && pos->numel() > 0;
  const c10::DeviceGuard g(dq.device());
  const int NH = nq + 2 * nkv;
  auto dqkv = at::empty({T, (long)NH * D}, dq.options());
  const long total = T * NH * (D / 16);
  if (total == 0) return dqkv;
  if (has_pos && pos->scalar_type() == at::kLong)
    hipLaunchKernelGGL(rope_bwd_kernel<int64_t>, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_ptr(dq),
                       bf_ptr(dk), bf_ptr(dv), cosT.data_ptr<float>(), sinT.data_ptr<float>(),
                       pos->data_ptr<int64_t>(), bf_mut(dqkv), nq, nkv, D, (int)seq_len, total);
  else
    hipLaunchKernelGGL(rope_bwd_kernel<int32_t>, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_ptr(dq),
                       bf_ptr(dk), bf_ptr(dv), cosT.data_ptr<float>(), sinT.data_ptr<float>(),
                       has_pos ? pos->data_ptr<int32_t>() : nullptr, bf_mut(dqkv), nq, nkv, D, (int)seq_len, total);
  return dqkv;
}

at::Tensor swiglu_fwd(const at::Tensor& gu) {
  LLMCTL_CHECK(gu.is_cuda() && gu.is_contiguous() && gu.scalar_type() == at::kBFloat16, "gu: contiguous bf16");
  const int F2 = gu.size(-1);
  LLMCTL_CHECK(F2 % 16 == 0, "2*ffn must be a multiple of 16");
  const int F = F2 / 2;
  const long T = gu.numel() / F2;
  const c10::DeviceGuard g(gu.device());
  auto sizes = gu.sizes().vec();
  sizes.back() = F;
  auto act = at::empty(sizes, gu.options());
  const long total = T * (F / 8);
  if (total)
    hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_ptr(gu), bf_mut(act), F,
                       total);
  return act;
}

at::Tensor swiglu_bwd(const at::Tensor& dact, const at::Tensor& gu) {
  LLMCTL_CHECK(dact.is_contiguous() && gu.is_contiguous(), "swiglu_bwd: contiguous inputs");
  const int F2 = gu.size(-1);
  const int F = F2 / 2;
  const long T = gu.numel() / F2;
  LLMCTL_CHECK(dact.numel() == T * F, "dact shape");
  const c10::DeviceGuard g(gu.device());
  auto dgu = at::empty_like(gu);
  const long total = T * (F / 8);
  if (total)
    hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(blocks_for(total)), dim3(256), 0, stream(), bf_ptr(dact), bf_ptr(gu),
                       bf_mut(dgu), F, total);
  return dgu;
}

at::Tensor gelu_fwd(const at::Tensor& x) {
  LLMCTL_CHECK(x.is_contiguous() && x.scalar_type() == at::kBFloat16 && x.numel() % 8 == 0, "gelu: bf16, numel%8");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  const long n8 = x.numel() / 8;
  if (n8) hipLaunchKernelGGL(gelu_fwd_kernel, dim3(blocks_for(n8)), dim3(256), 0, stream(), bf_ptr(x), bf_mut(y), n8);
  return y;
}

at::Tensor gelu_bwd(const at::Tensor& dy, const at::Tensor& x) {
  LLMCTL_CHECK(dy.is_contiguous() && x.is_contiguous() && dy.numel() == x.numel(), "gelu_bwd shapes");
  const c10::DeviceGuard g(x.device());
  auto dx = at::empty_like(x);
  const long n8 = x.numel() / 8;
  if (n8)
    hipLaunchKernelGGL(gelu_bwd_kernel, dim3(blocks_for(n8)), dim3(256), 0, stream(), bf_ptr(dy), bf_ptr(x), bf_mut(dx),
                       n8);
  return dx;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("rope_qkv_fwd", &rope_qkv_fwd);
  m.impl("rope_qk_inplace_", &rope_qk_inplace_);
  m.impl("rope_qkv_cache_fwd", &rope_qkv_cache_fwd);
  m.impl("rope_qkv_bwd", &rope_qkv_bwd);
  m.impl("swiglu_fwd", &swiglu_fwd);
  m.impl("swiglu_bwd", &swiglu_bwd);
  m.impl("gelu_fwd", &gelu_fwd);
  m.impl("gelu_bwd", &gelu_bwd);
}

}  // namespace llmctl
