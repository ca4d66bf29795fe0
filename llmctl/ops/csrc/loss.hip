// Fused softmax cross-entropy (gfx950).
//
// Forward: one 256-thread block per token row, single pass over the [V] bf16 logits with
// an online (max, sum-exp) per lane, combined across lanes/waves -> per-row loss and
// logsumexp (fp32).  No [T, V] fp32 softmax is ever materialised.
// Backward: dlogits = (softmax - onehot) * dloss, recomputed from logits + lse and written
// IN PLACE over the logits (they are dead after the loss), so the lm_head backward GEMM
// reads it directly and the [T, V] buffer is allocated once.
#include "common.h"

namespace llmctl {
namespace {

__device__ __forceinline__ void combine(float& m, float& s, float m2, float s2) {
  const float M = fmaxf(m, m2);
  if (M == -INFINITY) return;
  s = s * __expf(m - M) + s2 * __expf(m2 - M);
  m = M;
}

__global__ __launch_bounds__(256) void ce_fwd_kernel(const unsigned short* __restrict__ logits,
                                                      const int64_t* __restrict__ labels, float* __restrict__ loss,
                                                      float* __restrict__ lse_out, int V, long ignore_index) {
  __shared__ float sm[4], ss[4];
  const long row = blockIdx.x;
  const unsigned short* lr = logits + row * (long)V;
  float m = -INFINITY, s = 0.f;
  const int V8 = V & ~7;
  for (int c = threadIdx.x * 8; c < V8; c += 2048) {
    float v[8];
    load8(lr + c, v);
    float mx = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) mx = fmaxf(mx, v[j]);
    if (mx > m) {
      s = (m == -INFINITY) ? 0.f : s * __expf(m - mx);
      m = mx;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(v[j] - m);
  }
  for (int c = V8 + threadIdx.x; c < V; c += 256) {
    const float x = bf2f(lr[c]);
    if (x > m) {
      s = (m == -INFINITY) ? 0.f : s * __expf(m - x);
      m = x;
    }
    s += __expf(x - m);
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const float m2 = __shfl_xor(m, o), s2 = __shfl_xor(s, o);
    combine(m, s, m2, s2);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[w] = m;
    ss[w] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0], S = ss[0];
    for (int i = 1; i < 4; ++i) combine(M, S, sm[i], ss[i]);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const long lab = labels[row];
    loss[row] = (lab == ignore_index || lab < 0 || lab >= V) ? 0.f : lse - bf2f(lr[lab]);
  }
}

__global__ __launch_bounds__(256) void ce_bwd_kernel(const float* __restrict__ dloss,
                                                      const unsigned short* __restrict__ logits,
                                                      const float* __restrict__ lse,
                                                      const int64_t* __restrict__ labels,
                                                      unsigned short* __restrict__ out, int V, long ignore_index) {
  const long row = blockIdx.x;
  const long lab = labels[row];
  const bool valid = !(lab == ignore_index || lab < 0 || lab >= V);
  const float d = valid ? dloss[row] : 0.f;
  const float L = lse[row];
  const unsigned short* lr = logits + row * (long)V;
  unsigned short* orow = out + row * (long)V;
  const int V8 = V & ~7;
  for (int c = threadIdx.x * 8; c < V8; c += 2048) {
    float v[8];
    load8(lr + c, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      v[j] = __expf(v[j] - L) * d;
      if (c + j == lab) v[j] -= d;
    }
    store8(orow + c, v);
  }
  for (int c = V8 + threadIdx.x; c < V; c += 256) {
    float g = __expf(bf2f(lr[c]) - L) * d;
    if (c == lab) g -= d;
    orow[c] = f2bf(g);
  }
}

}  // namespace

std::tuple<at::Tensor, at::Tensor> cross_entropy_fwd(const at::Tensor& logits, const at::Tensor& labels,
                                                     int64_t ignore_index) {
  LLMCTL_CHECK(logits.is_cuda() && logits.dim() == 2 && logits.is_contiguous() &&
                   logits.scalar_type() == at::kBFloat16,
               "logits must be contiguous [T, V] bf16");
  LLMCTL_CHECK(labels.numel() == logits.size(0) && labels.scalar_type() == at::kLong && labels.is_contiguous(),
               "labels must be contiguous int64 [T]");
  const c10::DeviceGuard g(logits.device());
  const long T = logits.size(0);
  const int V = logits.size(1);
  auto loss = at::empty({T}, logits.options().dtype(at::kFloat));
  auto lse = at::empty({T}, logits.options().dtype(at::kFloat));
  if (T)
    hipLaunchKernelGGL(ce_fwd_kernel, dim3(T), dim3(256), 0, stream(), bf_ptr(logits), labels.data_ptr<int64_t>(),
                       loss.data_ptr<float>(), lse.data_ptr<float>(), V, (long)ignore_index);
  return {loss, lse};
}

at::Tensor cross_entropy_bwd(const at::Tensor& dloss, const at::Tensor& logits, const at::Tensor& lse,
                             const at::Tensor& labels, int64_t ignore_index, bool inplace) {
  LLMCTL_CHECK(dloss.scalar_type() == at::kFloat && dloss.is_contiguous() && dloss.numel() == logits.size(0),
               "dloss must be contiguous fp32 [T]");
  const c10::DeviceGuard g(logits.device());
  const long T = logits.size(0);
  const int V = logits.size(1);
  at::Tensor out = inplace ? logits : at::empty_like(logits);
  if (T)
    hipLaunchKernelGGL(ce_bwd_kernel, dim3(T), dim3(256), 0, stream(), dloss.data_ptr<float>(), bf_ptr(logits),
                       lse.data_ptr<float>(), labels.data_ptr<int64_t>(), bf_mut(out), V, (long)ignore_index);
  return out;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("cross_entropy_fwd", &cross_entropy_fwd);
  m.impl("cross_entropy_bwd", &cross_entropy_bwd);
}

}  // namespace llmctl
