// RMSNorm / LayerNorm forward+backward with fused residual add (gfx950).
//
// Memory-bound.  Layout: one wave64 per row, each lane owns 8 contiguous columns of every
// 512-column chunk (16-byte bf16x8 loads, fully coalesced 1 KiB per wave-instruction); the
// row lives in registers between the reduction and the normalised write, so x is read
// once.  Backward accumulates dW/dB per lane across the rows a wave visits, reduces the
// 4 waves of a block through LDS, writes one fp32 partial row per block, and a second tiny
// kernel sums the partials (no float atomics -> bitwise reproducible).
//
// Replaces: the reference's HF RMSNorm (library op, SURVEY §2.5 "fused_rmsnorm" declared
// plugin name, USER_GUIDE.md:268).
#include "common.h"

namespace llmctl {
namespace {

constexpr int kWaves = 4;  // 256-thread blocks

template <int NV, bool LN, bool ADD>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const unsigned short* __restrict__ x,
                                                        const unsigned short* __restrict__ res,
                                                        const unsigned short* __restrict__ w,
                                                        const unsigned short* __restrict__ b,
                                                        unsigned short* __restrict__ y,
                                                        unsigned short* __restrict__ res_out,
                                                        float* __restrict__ mu_out, float* __restrict__ rstd_out,
                                                        int T, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * kWaves;
  const float invH = 1.f / (float)H;
  for (int row = wave; row < T; row += nwaves) {
    const size_t base = (size_t)row * H;
    float v[NV][8];
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        load8(x + base + col, v[i]);
        if constexpr (ADD) {
          float r[8];
          load8(res + base + col, r);
          bf16x8 o;
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            o[j] = f2bf(v[i][j] + r[j]);
            v[i][j] = bf2f(o[j]);  // normalise the rounded residual (matches the oracle)
          }
          *reinterpret_cast<bf16x8*>(res_out + base + col) = o;
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) s += LN ? v[i][j] : v[i][j] * v[i][j];
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[i][j] = 0.f;
      }
    }
    float mean = 0.f, rs;
    if constexpr (LN) {
      mean = wave_sum(s) * invH;
      float ss = 0.f;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        const int col = i * 512 + lane * 8;
        if (col < H) {
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const float d = v[i][j] - mean;
            ss += d * d;
          }
        }
      }
      rs = rsqrtf(wave_sum(ss) * invH + eps);
    } else {
      rs = rsqrtf(wave_sum(s) * invH + eps);
    }
    if (lane == 0) {
      rstd_out[row] = rs;
      if constexpr (LN) mu_out[row] = mean;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        float wf[8], o[8];
        load8(w + col, wf);
        if constexpr (LN) {
          float bf[8];
          load8(b + col, bf);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rs * wf[j] + bf[j];
        } else {
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rs * wf[j];
        }
        store8(y + base + col, o);
      }
    }
  }
}

// RMSNorm statistics only: rstd[row] = rsqrt(mean(x[row]^2) + eps), one wave per row (serving
// prefill with the norm folded into the next projection: the GEMM scales its output rows by rstd
// and the norm weight lives in its K columns, so no normalised copy of x is written)
template <int NV>
__global__ __launch_bounds__(256) void rstd_kernel(const unsigned short* __restrict__ x, float* __restrict__ rstd_out,
                                                   int T, int H, float eps) {
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * kWaves + (threadIdx.x >> 6);
  const int nwaves = gridDim.x * kWaves;
  for (int row = wave; row < T; row += nwaves) {
    const size_t base = (size_t)row * H;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        float v[8];
        load8(x + base + col, v);
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[j] * v[j];
      }
    }
    s = wave_sum(s);
    if (lane == 0) rstd_out[row] = rsqrtf(s / (float)H + eps);
  }
}

template <int NV, bool LN, bool DRES>
__global__ __launch_bounds__(256, LN ? 1 : 2) void norm_bwd_kernel(const unsigned short* __restrict__ dy,
                                                                    const unsigned short* __restrict__ x,
                                                                    const unsigned short* __restrict__ w,
                                                                    const float* __restrict__ mu,
                                                                    const float* __restrict__ rstd,
                                                                    const unsigned short* __restrict__ dres,
                                                                    unsigned short* __restrict__ dx,
                                                                    float* __restrict__ dw_part,
                                                                    float* __restrict__ db_part, int T, int H) {
  // * software-pipelined over the wave's rows: the next row's x / dy (raw bf16) are in
  //   flight while the current row is reduced and written (HBM latency, not bandwidth, bounded
  //   the one-row-at-a-time form at ~2.9 TB/s);
  // * the per-column dW (dB) sums live in a wave-private LDS slab (float4 read-modify-write per
  //   row), not in 64 accumulator registers per lane, so two blocks fit per CU (RMSNorm).
  constexpr int W = NV * 512;
  __shared__ __attribute__((aligned(16))) float acc[(LN ? 2 : 1) * kWaves * W];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wave = blockIdx.x * kWaves + wid;
  const int nwaves = gridDim.x * kWaves;
  const float invH = 1.f / (float)H;
  float4* dwl = reinterpret_cast<float4*>(acc + wid * W);              // this wave's dW slab
  float4* dbl = reinterpret_cast<float4*>(acc + (kWaves + wid) * W);   // (LN) dB slab
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c4 = (i * 512 + lane * 8) / 4;
    dwl[c4] = dwl[c4 + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
    if constexpr (LN) dbl[c4] = dbl[c4 + 1] = make_float4(0.f, 0.f, 0.f, 0.f);
  }

  bf16x8 xr[NV], gr[NV], dr[DRES ? NV : 1];
  float r = 0.f, m = 0.f;
  auto fetch = [&](int row, bf16x8* xo, bf16x8* go, float& ro, float& mo) {
    const int rr = min(row, T - 1);  // unconditional (clamped) loads: no branch around them
    const size_t base = (size_t)rr * H;
    ro = rstd[rr];
    if constexpr (LN) mo = mu[rr];
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = min(i * 512 + lane * 8, H - 8);
      xo[i] = *reinterpret_cast<const bf16x8*>(x + base + col);
      go[i] = *reinterpret_cast<const bf16x8*>(dy + base + col);
    }
  };
  if (wave < T) fetch(wave, xr, gr, r, m);
  for (int row = wave; row < T; row += nwaves) {
    const size_t base = (size_t)row * H;
    if constexpr (DRES) {  // consumed by the second pass: the reductions cover its latency
#pragma unroll
      for (int i = 0; i < NV; ++i)
        dr[i] = *reinterpret_cast<const bf16x8*>(dres + base + min(i * 512 + lane * 8, H - 8));
    }
    bf16x8 xn[NV], gn[NV];
    float rn = 0.f, mn = 0.f;
    fetch(row + nwaves, xn, gn, rn, mn);
    float dot = 0.f, gs = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        float wf[8], pw[8], pb[8];
        load8(w + col, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (bf2f(xr[i][j]) - m) * r;
          const float dyf = bf2f(gr[i][j]);
          const float g = dyf * wf[j];
          dot += g * xh;
          gs += g;
          pw[j] = dyf * xh;
          pb[j] = dyf;
        }
        const int c4 = col / 4;
        float4 a0 = dwl[c4], a1 = dwl[c4 + 1];
        dwl[c4] = make_float4(a0.x + pw[0], a0.y + pw[1], a0.z + pw[2], a0.w + pw[3]);
        dwl[c4 + 1] = make_float4(a1.x + pw[4], a1.y + pw[5], a1.z + pw[6], a1.w + pw[7]);
        if constexpr (LN) {
          float4 b0 = dbl[c4], b1 = dbl[c4 + 1];
          dbl[c4] = make_float4(b0.x + pb[0], b0.y + pb[1], b0.z + pb[2], b0.w + pb[3]);
          dbl[c4 + 1] = make_float4(b1.x + pb[4], b1.y + pb[5], b1.z + pb[6], b1.w + pb[7]);
        }
      }
    }
    const float mdot = wave_sum(dot) * invH;
    const float mg = LN ? wave_sum(gs) * invH : 0.f;
    // re-expand the packed row in the second pass (no 2 x 64 live fp32 values across the
    // reductions: hipcc would otherwise keep the first pass's conversions and spill)
#pragma unroll
    for (int i = 0; i < NV; ++i) asm volatile("" : "+v"(xr[i]), "+v"(gr[i]));
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        float wf[8], o[8];
        load8(w + col, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float xh = (bf2f(xr[i][j]) - m) * r;
          o[j] = r * (bf2f(gr[i][j]) * wf[j] - mg - xh * mdot);
          if constexpr (DRES) o[j] += bf2f(dr[i][j]);
        }
        store8(dx + base + col, o);
      }
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      xr[i] = xn[i];
      gr[i] = gn[i];
    }
    r = rn;
    m = mn;
  }
  // block-reduce the 4 wave slabs: one fp32 partial row per block (no float atomics)
  __syncthreads();
#pragma unroll
  for (int pass = 0; pass < (LN ? 2 : 1); ++pass) {
    float* out = pass == 0 ? dw_part : db_part;
    const float* slab = acc + pass * kWaves * W;
    for (int c = threadIdx.x; c < H; c += 256) {
      float s = 0.f;
#pragma unroll
      for (int k = 0; k < kWaves; ++k) s += slab[k * W + c];
      out[(size_t)blockIdx.x * H + c] = s;
    }
  }
}

// rows wider than 4096: one row at a time, fp32 row in registers (the pipelined form spills)
template <int NV, bool LN, bool DRES>
__global__ __launch_bounds__(256) void norm_bwd_wide_kernel(const unsigned short* __restrict__ dy,
                                                        const unsigned short* __restrict__ x,
                                                        const unsigned short* __restrict__ w,
                                                        const float* __restrict__ mu,
                                                        const float* __restrict__ rstd,
                                                        const unsigned short* __restrict__ dres,
                                                        unsigned short* __restrict__ dx,
                                                        float* __restrict__ dw_part, float* __restrict__ db_part,
                                                        int T, int H) {
  __shared__ float red[kWaves][512];
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int wave = blockIdx.x * kWaves + wid;
  const int nwaves = gridDim.x * kWaves;
  const float invH = 1.f / (float)H;
  float dwa[NV][8], dba[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) dwa[i][j] = dba[i][j] = 0.f;

  for (int row = wave; row < T; row += nwaves) {
    const size_t base = (size_t)row * H;
    const float r = rstd[row];
    const float m = LN ? mu[row] : 0.f;
    float xh[NV][8], g[NV][8];
    float dot = 0.f, gs = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        float xf[8], dyf[8], wf[8];
        load8(x + base + col, xf);
        load8(dy + base + col, dyf);
        load8(w + col, wf);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          xh[i][j] = (xf[j] - m) * r;
          g[i][j] = dyf[j] * wf[j];
          dot += g[i][j] * xh[i][j];
          gs += g[i][j];
          dwa[i][j] += dyf[j] * xh[i][j];
          dba[i][j] += dyf[j];
        }
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) xh[i][j] = g[i][j] = 0.f;
      }
    }
    const float mdot = wave_sum(dot) * invH;
    const float mg = LN ? wave_sum(gs) * invH : 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int col = i * 512 + lane * 8;
      if (col < H) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = r * (g[i][j] - mg - xh[i][j] * mdot);
        if constexpr (DRES) {
          float d[8];
          load8(dres + base + col, d);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += d[j];
        }
        store8(dx + base + col, o);
      }
    }
  }
  // block-reduce the per-lane dW (and dB) partials, one fp32 row per block
#pragma unroll
  for (int pass = 0; pass < (LN ? 2 : 1); ++pass) {
    float* out = pass == 0 ? dw_part : db_part;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][lane * 8 + j] = pass == 0 ? dwa[i][j] : dba[i][j];
      __syncthreads();
      for (int c = threadIdx.x; c < 512; c += 256) {
        const int col = i * 512 + c;
        if (col < H) {
          float s = 0.f;
#pragma unroll
          for (int k = 0; k < kWaves; ++k) s += red[k][c];
          out[(size_t)blockIdx.x * H + col] = s;
        }
      }
      __syncthreads();
    }
  }
}


// sum partial rows [P, H] -> out[H] (bf16).  Block = 64 columns x 4 waves; wave w sums rows
// w, w+4, ... (4 independent loads in flight per lane), then the 4 waves combine via LDS.
__global__ __launch_bounds__(256) void col_reduce_kernel(const float* __restrict__ part, int P, int H,
                                                          unsigned short* __restrict__ out) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < H) {
    int p = w;
    for (; p + 12 < P; p += 16) {
      s0 += part[(size_t)p * H + c];
      s1 += part[(size_t)(p + 4) * H + c];
      s2 += part[(size_t)(p + 8) * H + c];
      s3 += part[(size_t)(p + 12) * H + c];
    }
    for (; p < P; p += 4) s0 += part[(size_t)p * H + c];
  }
  red[w][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (w == 0 && c < H) out[c] = f2bf(red[0][lane] + red[1][lane] + red[2][lane] + red[3][lane]);
}

int fwd_grid(int T) {
  int blocks = (T + kWaves - 1) / kWaves;
  return std::max(1, std::min(blocks, num_cus() * 8));
}

template <bool LN, bool ADD>
void launch_fwd(const at::Tensor& x, const at::Tensor* res, const at::Tensor& w, const at::Tensor* b,
                at::Tensor& y, at::Tensor* res_out, at::Tensor* mu, at::Tensor& rstd, double eps) {
  const int T = x.size(0), H = x.size(1);
  LLMCTL_CHECK(H % 8 == 0 && H <= 16384, "hidden size must be a multiple of 8 and <= 16384, got ", H);
  const int nv = (H + 511) / 512;
  dim3 grid(fwd_grid(T)), block(256);
  auto s = stream();
#define LAUNCH(NV)                                                                                           \
  hipLaunchKernelGGL((norm_fwd_kernel<NV, LN, ADD>), grid, block, 0, s, bf_ptr(x),                         \
                     res ? bf_ptr(*res) : nullptr, bf_ptr(w), b ? bf_ptr(*b) : nullptr, bf_mut(y),            \
                     res_out ? bf_mut(*res_out) : nullptr, mu ? mu->data_ptr<float>() : nullptr,              \
                     rstd.data_ptr<float>(), T, H, (float)eps)
  switch (nv) {
    case 1: LAUNCH(1); break;
    case 2: LAUNCH(2); break;
    case 3: LAUNCH(3); break;
    case 4: LAUNCH(4); break;
    case 5: case 6: LAUNCH(6); break;
    case 7: case 8: LAUNCH(8); break;
    case 9: case 10: case 11: case 12: LAUNCH(12); break;
    default: LAUNCH(16); break;
  }
#undef LAUNCH
}

template <bool LN>
void launch_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w, const at::Tensor* mu,
                const at::Tensor& rstd, const c10::optional<at::Tensor>& dres, at::Tensor& dx, at::Tensor& dw,
                at::Tensor* db) {
  const int T = x.size(0), H = x.size(1);
  const int nv = (H + 511) / 512;
  // pipelined kernel (H <= 4096): 2 blocks per CU for RMSNorm (LDS dW slabs, 64 KB each)
  const int per_cu = (nv <= 8 && !LN) ? 2 : 1;
  const int grid = std::max(1, std::min((T + kWaves - 1) / kWaves, per_cu * num_cus()));
  auto opts = x.options().dtype(at::kFloat);
  at::Tensor dw_part = at::empty({grid, H}, opts);
  at::Tensor db_part = LN ? at::empty({grid, H}, opts) : at::Tensor();
  const bool has_dres = dres.has_value() && dres->defined();
  auto s = stream();
#define LAUNCH(NV)                                                                                         \
  if (has_dres)                                                                                            \
    hipLaunchKernelGGL((norm_bwd_kernel<NV, LN, true>), dim3(grid), dim3(256), 0, s, bf_ptr(dy), bf_ptr(x), \
                       bf_ptr(w), mu ? mu->data_ptr<float>() : nullptr, rstd.data_ptr<float>(),             \
                       bf_ptr(*dres), bf_mut(dx), dw_part.data_ptr<float>(),                                 \
                       LN ? db_part.data_ptr<float>() : nullptr, T, H);                                     \
  else                                                                                                     \
    hipLaunchKernelGGL((norm_bwd_kernel<NV, LN, false>), dim3(grid), dim3(256), 0, s, bf_ptr(dy), bf_ptr(x), \
                       bf_ptr(w), mu ? mu->data_ptr<float>() : nullptr, rstd.data_ptr<float>(), nullptr,     \
                       bf_mut(dx), dw_part.data_ptr<float>(), LN ? db_part.data_ptr<float>() : nullptr, T, H)
#define LAUNCHW(NV)                                                                                          \
  if (has_dres)                                                                                              \
    hipLaunchKernelGGL((norm_bwd_wide_kernel<NV, LN, true>), dim3(grid), dim3(256), 0, s, bf_ptr(dy),          \
                       bf_ptr(x), bf_ptr(w), mu ? mu->data_ptr<float>() : nullptr, rstd.data_ptr<float>(),    \
                       bf_ptr(*dres), bf_mut(dx), dw_part.data_ptr<float>(),                                   \
                       LN ? db_part.data_ptr<float>() : nullptr, T, H);                                       \
  else                                                                                                       \
    hipLaunchKernelGGL((norm_bwd_wide_kernel<NV, LN, false>), dim3(grid), dim3(256), 0, s, bf_ptr(dy),         \
                       bf_ptr(x), bf_ptr(w), mu ? mu->data_ptr<float>() : nullptr, rstd.data_ptr<float>(),    \
                       nullptr, bf_mut(dx), dw_part.data_ptr<float>(), LN ? db_part.data_ptr<float>() : nullptr, \
                       T, H)
  switch (nv) {
    case 1: LAUNCH(1); break;
    case 2: LAUNCH(2); break;
    case 3: LAUNCH(3); break;
    case 4: LAUNCH(4); break;
    case 5: case 6: LAUNCH(6); break;
    case 7: case 8: LAUNCH(8); break;
    case 9: case 10: case 11: case 12: LAUNCHW(12); break;
    default: LAUNCHW(16); break;
  }
#undef LAUNCH
#undef LAUNCHW
  hipLaunchKernelGGL(col_reduce_kernel, dim3((H + 63) / 64), dim3(256), 0, s, dw_part.data_ptr<float>(), grid, H,
                     bf_mut(dw));
  if (LN)
    hipLaunchKernelGGL(col_reduce_kernel, dim3((H + 63) / 64), dim3(256), 0, s, db_part.data_ptr<float>(), grid, H,
                       bf_mut(*db));
}

void check2d(const at::Tensor& t, const char* n) {
  LLMCTL_CHECK(t.is_cuda() && t.dim() == 2 && t.is_contiguous() && t.scalar_type() == at::kBFloat16, n,
               " must be a contiguous 2-D bf16 GPU tensor");
}

}  // namespace

std::tuple<at::Tensor, at::Tensor> rmsnorm_fwd(const at::Tensor& x, const at::Tensor& w, double eps) {
  check2d(x, "x");
  LLMCTL_CHECK(w.numel() == x.size(1) && w.scalar_type() == at::kBFloat16, "weight shape/dtype");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  auto rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  launch_fwd<false, false>(x, nullptr, w, nullptr, y, nullptr, nullptr, rstd, eps);
  return {y, rstd};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> add_rmsnorm_fwd(const at::Tensor& x, const at::Tensor& res,
                                                                const at::Tensor& w, double eps) {
  check2d(x, "x");
  check2d(res, "residual");
  LLMCTL_CHECK(x.sizes() == res.sizes(), "x/residual shape mismatch");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  auto ro = at::empty_like(x);
  auto rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  launch_fwd<false, true>(x, &res, w, nullptr, y, &ro, nullptr, rstd, eps);
  return {y, ro, rstd};
}

std::tuple<at::Tensor, at::Tensor> rmsnorm_bwd(const at::Tensor& dy, const at::Tensor& x, const at::Tensor& w,
                                               const at::Tensor& rstd, const c10::optional<at::Tensor>& dres) {
  check2d(dy, "dy");
  check2d(x, "x");
  if (dres.has_value() && dres->defined()) check2d(*dres, "dres");
  const c10::DeviceGuard g(x.device());
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(w);
  launch_bwd<false>(dy, x, w, nullptr, rstd, dres, dx, dw, nullptr);
  return {dx, dw};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> layernorm_fwd(const at::Tensor& x, const at::Tensor& w,
                                                              const at::Tensor& b, double eps) {
  check2d(x, "x");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  auto mu = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  launch_fwd<true, false>(x, nullptr, w, &b, y, nullptr, &mu, rstd, eps);
  return {y, mu, rstd};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor, at::Tensor> add_layernorm_fwd(const at::Tensor& x,
                                                                              const at::Tensor& res,
                                                                              const at::Tensor& w,
                                                                              const at::Tensor& b, double eps) {
  check2d(x, "x");
  check2d(res, "residual");
  const c10::DeviceGuard g(x.device());
  auto y = at::empty_like(x);
  auto ro = at::empty_like(x);
  auto mu = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  auto rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  launch_fwd<true, true>(x, &res, w, &b, y, &ro, &mu, rstd, eps);
  return {y, ro, mu, rstd};
}

std::tuple<at::Tensor, at::Tensor, at::Tensor> layernorm_bwd(const at::Tensor& dy, const at::Tensor& x,
                                                              const at::Tensor& w, const at::Tensor& mu,
                                                              const at::Tensor& rstd,
                                                              const c10::optional<at::Tensor>& dres) {
  check2d(dy, "dy");
  check2d(x, "x");
  const c10::DeviceGuard g(x.device());
  auto dx = at::empty_like(x);
  auto dw = at::empty_like(w);
  auto db = at::empty_like(w);
  launch_bwd<true>(dy, x, w, &mu, rstd, dres, dx, dw, &db);
  return {dx, dw, db};
}

at::Tensor rms_rstd(const at::Tensor& x, double eps) {
  check2d(x, "x");
  const int T = x.size(0), H = x.size(1);
  LLMCTL_CHECK(H % 8 == 0 && H <= 16384, "rms_rstd: hidden size must be a multiple of 8 and <= 16384, got ", H);
  const c10::DeviceGuard g(x.device());
  auto rstd = at::empty({x.size(0)}, x.options().dtype(at::kFloat));
  if (T == 0) return rstd;
  const int nv = (H + 511) / 512;
  dim3 grid(fwd_grid(T)), block(256);
  auto s = stream();
#define LAUNCH(NV) \
  hipLaunchKernelGGL((rstd_kernel<NV>), grid, block, 0, s, bf_ptr(x), rstd.data_ptr<float>(), T, H, (float)eps)
  switch (nv) {
    case 1: LAUNCH(1); break;
    case 2: LAUNCH(2); break;
    case 3: case 4: LAUNCH(4); break;
    case 5: case 6: case 7: case 8: LAUNCH(8); break;
    default: LAUNCH(32); break;
  }
#undef LAUNCH
  return rstd;
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("rms_rstd", &rms_rstd);
  m.impl("rmsnorm_fwd", &rmsnorm_fwd);
  m.impl("add_rmsnorm_fwd", &add_rmsnorm_fwd);
  m.impl("rmsnorm_bwd", &rmsnorm_bwd);
  m.impl("layernorm_fwd", &layernorm_fwd);
  m.impl("add_layernorm_fwd", &add_layernorm_fwd);
  m.impl("layernorm_bwd", &layernorm_bwd);
}

}  // namespace llmctl
