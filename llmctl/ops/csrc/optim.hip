// Fused AdamW over flat buffers + sum-of-squares reduction for gradient clipping (gfx950).
//
// AdamW: one launch per flat region (see llmctl/runtime/flat.py).  Per element it reads
// the bf16|fp32 grad, fp32 master, fp32 m and v (14-16 B) and writes master, m, v and the
// bf16 param (14 B) — ~28 B/param, HBM-bound by design; 8 elements per lane (16-B bf16 and
// 2×16-B fp32 vectors), grid-stride at ~8 blocks per CU.  Plain (cached) loads and stores:
// non-temporal ones measured 4.58 vs 5.85 TB/s (tools/adamw_bench.py, 2e9 elements, round 3).  The clip coefficient and the
// 1/world DP average arrive as a device scalar (grad_scale), so clipping needs no host
// synchronisation.  A non-finite scale skips the update (overflow skip-step policy).
//
// l2norm_sq_: grid-stride sum of squares, one wave shuffle + LDS reduction per block and ONE
// float atomic per block into the fp32 accumulator.
#include "common.h"

namespace llmctl {
namespace {

template <typename GT>
__device__ __forceinline__ void load_grad8(const GT* g, float* out);

template <>
__device__ __forceinline__ void load_grad8<unsigned short>(const unsigned short* g, float* out) {
  load8(g, out);
}
template <>
__device__ __forceinline__ void load_grad8<float>(const float* g, float* out) {
  *reinterpret_cast<float4*>(out) = reinterpret_cast<const float4*>(g)[0];
  *reinterpret_cast<float4*>(out + 4) = reinterpret_cast<const float4*>(g)[1];
}

template <typename GT>
__global__ __launch_bounds__(256) void adamw_kernel(unsigned short* __restrict__ param, float* __restrict__ master,
                                                     const GT* __restrict__ grad, float* __restrict__ m,
                                                     float* __restrict__ v, long n, float lr, float b1, float b2,
                                                     float eps, float wd, float inv_bc1, float inv_sqrt_bc2,
                                                     const float* __restrict__ gscale) {
  const float gs = gscale ? gscale[0] : 1.f;
  // non-finite grad scale (the optimizer passes NaN when the global grad norm overflowed):
  // skip the whole update — params, master and moments stay untouched on every rank
  if (!__builtin_isfinite(gs)) return;
  const float decay = 1.f - lr * wd;
  const float step = lr * inv_bc1;
  const long n8 = n >> 3;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    const long o = i * 8;
    float g[8], w[8], mm[8], vv[8];
    load_grad8<GT>(grad + o, g);
    *reinterpret_cast<float4*>(w) = reinterpret_cast<const float4*>(master + o)[0];
    *reinterpret_cast<float4*>(w + 4) = reinterpret_cast<const float4*>(master + o)[1];
    *reinterpret_cast<float4*>(mm) = reinterpret_cast<const float4*>(m + o)[0];
    *reinterpret_cast<float4*>(mm + 4) = reinterpret_cast<const float4*>(m + o)[1];
    *reinterpret_cast<float4*>(vv) = reinterpret_cast<const float4*>(v + o)[0];
    *reinterpret_cast<float4*>(vv + 4) = reinterpret_cast<const float4*>(v + o)[1];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float gj = g[j] * gs;
      mm[j] = b1 * mm[j] + (1.f - b1) * gj;
      vv[j] = b2 * vv[j] + (1.f - b2) * gj * gj;
      const float denom = sqrtf(vv[j]) * inv_sqrt_bc2 + eps;
      w[j] = w[j] * decay - step * mm[j] / denom;
    }
    reinterpret_cast<float4*>(master + o)[0] = *reinterpret_cast<float4*>(w);
    reinterpret_cast<float4*>(master + o)[1] = *reinterpret_cast<float4*>(w + 4);
    reinterpret_cast<float4*>(m + o)[0] = *reinterpret_cast<float4*>(mm);
    reinterpret_cast<float4*>(m + o)[1] = *reinterpret_cast<float4*>(mm + 4);
    reinterpret_cast<float4*>(v + o)[0] = *reinterpret_cast<float4*>(vv);
    reinterpret_cast<float4*>(v + o)[1] = *reinterpret_cast<float4*>(vv + 4);
    store8(param + o, w);
  }
  // scalar tail (n % 8) handled by block 0
  if (blockIdx.x == 0) {
    for (long o = n8 * 8 + threadIdx.x; o < n; o += 256) {
      float gj;
      if constexpr (sizeof(GT) == 2) gj = bf2f(((const unsigned short*)grad)[o]) * gs;
      else gj = ((const float*)grad)[o] * gs;
      const float mj = b1 * m[o] + (1.f - b1) * gj;
      const float vj = b2 * v[o] + (1.f - b2) * gj * gj;
      const float w = master[o] * decay - step * mj / (sqrtf(vj) * inv_sqrt_bc2 + eps);
      m[o] = mj;
      v[o] = vj;
      master[o] = w;
      param[o] = f2bf(w);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, long n, float* __restrict__ out) {
  __shared__ float sm[4];
  float s = 0.f;
  const long n8 = n >> 3;
  const long stride = (long)gridDim.x * 256;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n8; i += stride) {
    float v[8];
    load_grad8<T>(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) s += v[j] * v[j];
  }
  if (blockIdx.x == 0) {
    for (long o = n8 * 8 + threadIdx.x; o < n; o += 256) {
      float v;
      if constexpr (sizeof(T) == 2) v = bf2f(((const unsigned short*)x)[o]);
      else v = ((const float*)x)[o];
      s += v * v;
    }
  }
  const float r = block_sum<4>(s, sm);
  if (threadIdx.x == 0) atomicAdd(out, r);
}

int stream_grid(long n8) {
  long b = (n8 + 255) / 256;
  return (int)std::max(1L, std::min(b, (long)num_cus() * 8));
}

}  // namespace

void adamw_step_(at::Tensor& param, at::Tensor& master, const at::Tensor& grad, at::Tensor& exp_avg,
                 at::Tensor& exp_avg_sq, double lr, double beta1, double beta2, double eps, double weight_decay,
                 double bc1, double bc2, const c10::optional<at::Tensor>& grad_scale) {
  const long n = param.numel();
  LLMCTL_CHECK(param.scalar_type() == at::kBFloat16 && master.scalar_type() == at::kFloat &&
                   exp_avg.scalar_type() == at::kFloat && exp_avg_sq.scalar_type() == at::kFloat,
               "adamw dtypes: bf16 param, fp32 master/m/v");
  LLMCTL_CHECK(master.numel() == n && grad.numel() == n && exp_avg.numel() == n && exp_avg_sq.numel() == n,
               "adamw: size mismatch");
  LLMCTL_CHECK(param.is_contiguous() && master.is_contiguous() && grad.is_contiguous() && exp_avg.is_contiguous() &&
                   exp_avg_sq.is_contiguous(),
               "adamw: contiguous buffers required");
  // 16-byte alignment of every vector stream
  LLMCTL_CHECK((reinterpret_cast<uintptr_t>(param.data_ptr()) & 15) == 0 &&
                   (reinterpret_cast<uintptr_t>(master.data_ptr()) & 15) == 0,
               "adamw: buffers must be 16-byte aligned");
  if (n == 0) return;
  const c10::DeviceGuard g(param.device());
  const float* gs = nullptr;
  if (grad_scale.has_value() && grad_scale->defined()) {
    LLMCTL_CHECK(grad_scale->scalar_type() == at::kFloat && grad_scale->is_cuda(), "grad_scale: fp32 GPU scalar");
    gs = grad_scale->data_ptr<float>();
  }
  const int grid = stream_grid(n / 8 + 1);
  const float inv_bc1 = 1.f / (float)bc1, inv_sqrt_bc2 = 1.f / sqrtf((float)bc2);
  if (grad.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(adamw_kernel<unsigned short>, dim3(grid), dim3(256), 0, stream(), bf_mut(param),
                       master.data_ptr<float>(), bf_ptr(grad), exp_avg.data_ptr<float>(),
                       exp_avg_sq.data_ptr<float>(), n, (float)lr, (float)beta1, (float)beta2, (float)eps,
                       (float)weight_decay, inv_bc1, inv_sqrt_bc2, gs);
  else if (grad.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(adamw_kernel<float>, dim3(grid), dim3(256), 0, stream(), bf_mut(param),
                       master.data_ptr<float>(), grad.data_ptr<float>(), exp_avg.data_ptr<float>(),
                       exp_avg_sq.data_ptr<float>(), n, (float)lr, (float)beta1, (float)beta2, (float)eps,
                       (float)weight_decay, inv_bc1, inv_sqrt_bc2, gs);
  else
    LLMCTL_CHECK(false, "adamw: grad must be bf16 or fp32");
}

void l2norm_sq_(const at::Tensor& x, at::Tensor& out) {
  LLMCTL_CHECK(x.is_contiguous() && out.scalar_type() == at::kFloat && out.numel() >= 1, "l2norm_sq_ args");
  const long n = x.numel();
  if (n == 0) return;
  const c10::DeviceGuard g(x.device());
  const int grid = stream_grid(n / 8 + 1);
  if (x.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(sumsq_kernel<unsigned short>, dim3(grid), dim3(256), 0, stream(), bf_ptr(x), n,
                       out.data_ptr<float>());
  else if (x.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(sumsq_kernel<float>, dim3(grid), dim3(256), 0, stream(), x.data_ptr<float>(), n,
                       out.data_ptr<float>());
  else
    LLMCTL_CHECK(false, "l2norm_sq_: bf16 or fp32");
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("adamw_step_", &adamw_step_);
  m.impl("l2norm_sq_", &l2norm_sq_);
}

}  // namespace llmctl
