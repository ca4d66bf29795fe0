// Batched token sampling: temperature / top-k / top-p / greedy in one launch (gfx950).
//
// Replaces the reference's per-request Python loop with a host sync per token
// (``server.py:209-235``).  One 256-thread workgroup per sequence row; no sort: the top-k
// and top-p cut-offs are found by bisection on the logit threshold (count / probability
// mass of logits >= T are monotone in T), then an inverse-CDF draw over the kept tokens in
// index order using a caller-provided uniform (so results are reproducible and the whole
// step is hipGraph-capturable: no RNG state, no allocation, no host sync).
#include "common.h"

namespace llmctl {
namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p, long i);
template <>
__device__ __forceinline__ float ld<unsigned short>(const unsigned short* p, long i) { return bf2f(p[i]); }
template <>
__device__ __forceinline__ float ld<float>(const float* p, long i) { return p[i]; }

__device__ __forceinline__ float bmax(float v, float* sm) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) sm[w] = v;
  __syncthreads();
  float r = fmaxf(fmaxf(sm[0], sm[1]), fmaxf(sm[2], sm[3]));
  __syncthreads();
  return r;
}

template <typename T>
__global__ __launch_bounds__(256) void sample_kernel(const T* __restrict__ logits, const float* __restrict__ temp,
                                                      const int* __restrict__ topk, const float* __restrict__ topp,
                                                      const float* __restrict__ uni, int64_t* __restrict__ out, int V) {
  __shared__ float sm[8];
  __shared__ float scan[256];
  __shared__ int found;
  const long row = blockIdx.x;
  const T* lr = logits + row * (long)V;
  const int tid = threadIdx.x;
  const float t = temp[row];
  if (t <= 0.f) {  // greedy: argmax, lowest index on ties
    float best = -INFINITY;
    int bi = 0x7fffffff;
    int i0 = 0;
    if constexpr (sizeof(T) == 2) {
      // 16-B vectors (8 logits per lane, 4 loads in flight per unrolled step): a 32k-vocab row
      // is 16 vector steps per thread instead of 125 dependent scalar loads (37 -> a few us)
      if ((V & 7) == 0 && (reinterpret_cast<uintptr_t>(lr) & 15) == 0) {
        const bf16x8* lv = reinterpret_cast<const bf16x8*>(lr);
        const int V8 = V >> 3;
#pragma unroll 4
        for (int c = tid; c < V8; c += 256) {
          const bf16x8 v = lv[c];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float x = bf2f(v[e]);
            if (x > best) {  // in index order within the thread: strict > keeps the lowest index
              best = x;
              bi = c * 8 + e;
            }
          }
        }
        i0 = V;
      }
    }
    for (int i = i0 + tid; i < V; i += 256) {
      const float x = ld(lr, i);
      if (x > best) {
        best = x;
        bi = i;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o);
      const int oi = __shfl_xor(bi, o);
      if (ob > best || (ob == best && oi < bi)) {
        best = ob;
        bi = oi;
      }
    }
    __shared__ float wb[4];
    __shared__ int wi[4];
    if ((tid & 63) == 0) {
      wb[tid >> 6] = best;
      wi[tid >> 6] = bi;
    }
    __syncthreads();
    if (tid == 0) {
      float B = wb[0];
      int I = wi[0];
      for (int w = 1; w < 4; ++w)
        if (wb[w] > B || (wb[w] == B && wi[w] < I)) {
          B = wb[w];
          I = wi[w];
        }
      out[row] = I;
    }
    return;
  }
  const float inv_t = 1.f / t;
  // max / min of scaled logits
  float mx = -INFINITY, mn = INFINITY;
  for (int i = tid; i < V; i += 256) {
    const float x = ld(lr, i) * inv_t;
    mx = fmaxf(mx, x);
    mn = fminf(mn, x);
  }
  mx = bmax(mx, sm);
  mn = -bmax(-mn, sm);
  float z = 0.f;
  for (int i = tid; i < V; i += 256) z += __expf(ld(lr, i) * inv_t - mx);
  z = block_sum<4>(z, sm);
  float thr = -INFINITY;
  const int k = topk[row];
  if (k > 0 && k < V) {  // largest T with count(x >= T) >= k
    float lo = mn, hi = mx + 1e-6f;
    for (int it = 0; it < 40; ++it) {
      const float mid = 0.5f * (lo + hi);
      float c = 0.f;
      for (int i = tid; i < V; i += 256) c += (ld(lr, i) * inv_t >= mid) ? 1.f : 0.f;
      c = block_sum<4>(c, sm);
      if (c >= (float)k) lo = mid;
      else hi = mid;
    }
    thr = lo;
  }
  const float p = topp[row];
  if (p < 1.f) {  // largest T with mass(x >= T) >= p
    float lo = mn, hi = mx + 1e-6f;
    const float target = p * z;
    for (int it = 0; it < 40; ++it) {
      const float mid = 0.5f * (lo + hi);
      float s = 0.f;
      for (int i = tid; i < V; i += 256) {
        const float x = ld(lr, i) * inv_t;
        if (x >= mid) s += __expf(x - mx);
      }
      s = block_sum<4>(s, sm);
      if (s >= target) lo = mid;
      else hi = mid;
    }
    thr = fmaxf(thr, lo);
  }
  // inverse CDF over kept tokens in index order: contiguous chunk per thread
  const int chunk = (V + 255) / 256;
  const int c0 = tid * chunk, c1 = min(V, c0 + chunk);
  float cs = 0.f;
  for (int i = c0; i < c1; ++i) {
    const float x = ld(lr, i) * inv_t;
    if (x >= thr) cs += __expf(x - mx);
  }
  scan[tid] = cs;
  if (tid == 0) found = -1;
  __syncthreads();
  if (tid == 0) {  // exclusive scan (256 elements, serial: negligible vs the passes above)
    float acc = 0.f;
    for (int i = 0; i < 256; ++i) {
      const float v = scan[i];
      scan[i] = acc;
      acc += v;
    }
    sm[4] = acc;
  }
  __syncthreads();
  const float r = uni[row] * sm[4];
  float acc = scan[tid];
  if (acc <= r && acc + cs > r) {
    for (int i = c0; i < c1; ++i) {
      const float x = ld(lr, i) * inv_t;
      if (x >= thr) {
        acc += __expf(x - mx);
        if (acc > r) {  // chunks are disjoint and ordered: exactly one thread gets here
          found = i;
          break;
        }
      }
    }
  }
  __syncthreads();
  if (tid == 0) {
    int f = found;
    if (f < 0) {  // r at the very top (rounding): last kept token
      for (int i = V - 1; i >= 0; --i)
        if (ld(lr, i) * inv_t >= thr) {
          f = i;
          break;
        }
    }
    out[row] = f < 0 ? 0 : f;
  }
}

}  // namespace

at::Tensor sample(const at::Tensor& logits, const at::Tensor& temperature, const at::Tensor& top_k,
                  const at::Tensor& top_p, const at::Tensor& uniform) {
  LLMCTL_CHECK(logits.dim() == 2 && logits.is_contiguous(), "logits: contiguous [N, V]");
  const int N = logits.size(0), V = logits.size(1);
  LLMCTL_CHECK(temperature.scalar_type() == at::kFloat && top_p.scalar_type() == at::kFloat &&
                   uniform.scalar_type() == at::kFloat && top_k.scalar_type() == at::kInt,
               "temperature/top_p/uniform fp32, top_k int32");
  LLMCTL_CHECK(temperature.numel() == N && top_k.numel() == N && top_p.numel() == N && uniform.numel() == N,
               "per-row parameter tensors must have N elements");
  const c10::DeviceGuard g(logits.device());
  auto out = at::empty({N}, logits.options().dtype(at::kLong));
  if (N == 0) return out;
  if (logits.scalar_type() == at::kBFloat16)
    hipLaunchKernelGGL(sample_kernel<unsigned short>, dim3(N), dim3(256), 0, stream(), bf_ptr(logits),
                       temperature.data_ptr<float>(), top_k.data_ptr<int>(), top_p.data_ptr<float>(),
                       uniform.data_ptr<float>(), out.data_ptr<int64_t>(), V);
  else if (logits.scalar_type() == at::kFloat)
    hipLaunchKernelGGL(sample_kernel<float>, dim3(N), dim3(256), 0, stream(), logits.data_ptr<float>(),
                       temperature.data_ptr<float>(), top_k.data_ptr<int>(), top_p.data_ptr<float>(),
                       uniform.data_ptr<float>(), out.data_ptr<int64_t>(), V);
  else
    LLMCTL_CHECK(false, "logits must be bf16 or fp32");
  return out;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("sample", &sample); }

}  // namespace llmctl
