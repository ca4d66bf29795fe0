// One-shot all-reduce over xGMI peer memory for small tensor-parallel messages (gfx950).
//
// RCCL's ring/tree all-reduce pays several link latencies per call, which dominates the
// per-layer TP all-reduces of decode (a few KB to ~1 MB).  With all ranks of a node mapped
// into each other's address space (hipIpc* over the xGMI fabric), one kernel does it in one
// step:
//   1. block b copies its slice of the input into this rank's IPC data buffer (half = epoch
//      parity, so a call never overwrites what a slow peer may still read from the last one);
//   2. block b stores the epoch into flag[b][rank] of every peer (system-scope release) and
//      spins on its own flag[b][*] (system-scope acquire, bounded: a timeout sets an error
//      word instead of hanging the GPU);
//   3. block b sums its slice over all peers' buffers (fp32) and writes the output.
// Per-block flags mean no grid-wide barrier.  The epoch lives in device memory and is bumped
// by the last block to finish, so the kernel is hipGraph-capturable (no host arguments
// change between calls).  Data and flag buffers are allocated uncached
// (hipDeviceMallocUncached): remote reads always see the writer's memory.
#include "common.h"

#include <cstring>

namespace llmctl {
namespace {

constexpr int CAR_MAX_RANKS = 8;
constexpr int CAR_MAX_BLOCKS = 64;
// signal buffer layout (uint32): flags[CAR_MAX_BLOCKS][CAR_MAX_RANKS] (one-shot, and the two-shot
// kernel's first round), flags2[...] (the two-shot kernel's second round), then epoch, done, error
constexpr int CAR_FLAGS2 = CAR_MAX_BLOCKS * CAR_MAX_RANKS;
constexpr int CAR_EPOCH = 2 * CAR_MAX_BLOCKS * CAR_MAX_RANKS;
constexpr int CAR_DONE = CAR_EPOCH + 1;
constexpr int CAR_ERROR = CAR_EPOCH + 2;
constexpr int CAR_SIG_WORDS = CAR_EPOCH + 16;

struct CarArgs {
  const unsigned short* inp;
  unsigned short* out;
  unsigned long long data[CAR_MAX_RANKS];  // per-rank data buffers (this process's mappings)
  unsigned long long sig[CAR_MAX_RANKS];   // per-rank signal buffers
  int rank, world;
  long n8;          // number of 8-element (16-B) vectors
  long half_elems;  // elements per epoch-parity half of a data buffer
};

// step 2 (signal + bounded wait for this block's flags, in flag array `round`) shared by the kernels
__device__ __forceinline__ void car_signal_wait(const CarArgs& a, unsigned* my_sig, int b, int tid, unsigned epoch,
                                                int round = 0) {
  if (tid < a.world) {
    const int fo = round * CAR_FLAGS2;
    unsigned* peer = reinterpret_cast<unsigned*>(a.sig[tid]);
    __hip_atomic_store(peer + fo + b * CAR_MAX_RANKS + a.rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* f = my_sig + fo + b * CAR_MAX_RANKS + tid;
    long spins = 0;
    // wrap-aware: a peer already one epoch ahead may have overwritten this flag with epoch + 1
    // (it finished epoch `epoch` after seeing our signal, before we read its) -- that counts too
    while ((int)(__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) - epoch) < 0) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1L << 26)) {  // ~seconds: a peer is gone; report instead of hanging
        __hip_atomic_store(my_sig + CAR_ERROR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
}

// step 4: the last block to finish advances the epoch (device-side: graph replays stay correct)
__device__ __forceinline__ void car_finish(unsigned* my_sig, int nb, int tid, unsigned epoch) {
  __syncthreads();
  if (tid == 0) {
    const unsigned d = __hip_atomic_fetch_add(my_sig + CAR_DONE, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned)nb - 1) {
      __hip_atomic_store(my_sig + CAR_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(my_sig + CAR_EPOCH, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

__device__ __forceinline__ unsigned car_epoch(unsigned* my_sig, int tid) {
  __shared__ unsigned s_epoch;
  if (tid == 0) s_epoch = __hip_atomic_load(my_sig + CAR_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  return s_epoch;
}

__global__ __launch_bounds__(256) void car_oneshot_kernel(CarArgs a) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  unsigned* my_sig = reinterpret_cast<unsigned*>(a.sig[a.rank]);
  const unsigned epoch = car_epoch(my_sig, tid);
  const long par = (long)(epoch & 1) * a.half_elems;
  // 1. input slice -> own buffer
  uint4* mine = reinterpret_cast<uint4*>(reinterpret_cast<unsigned short*>(a.data[a.rank]) + par);
  const uint4* in = reinterpret_cast<const uint4*>(a.inp);
  for (long i = (long)b * 256 + tid; i < a.n8; i += (long)nb * 256) mine[i] = in[i];
  __threadfence_system();
  __syncthreads();
  // 2. signal every peer, then wait for every peer's signal for this block
  car_signal_wait(a, my_sig, b, tid, epoch);
  // 3. reduce this block's slice over all ranks
  for (long i = (long)b * 256 + tid; i < a.n8; i += (long)nb * 256) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int r = 0; r < a.world; ++r) {
      using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
      const u32x4* src = reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned short*>(a.data[r]) + par);
      const u32x4 v = __builtin_nontemporal_load(src + i);
      const unsigned short* h = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(h[j]);
    }
    store8(a.out + i * 8, acc);
  }
  car_finish(my_sig, nb, tid, epoch);
}

// Two-shot all-reduce for prefill-sized messages (MBs): the one-shot kernel reads (world - 1) x n
// bytes from peers per rank; here rank r first reduces only its 1/world slice (reading (world-1)/
// world x n), publishes it, and then gathers the other ranks' reduced slices (another (world-1)/
// world x n) — 2 (world-1)/world x n per rank, the ring's byte count, in two flag rounds.  Slice s
// is cut into nb sub-ranges; block b owns sub-range b of every slice on every rank, so the per-
// block flags of round 0 (everyone's copy of sub-range b landed) and round 1 (everyone's reduced
// sub-range b landed) need no grid barrier.  Buffer half = [input copy | reduced slice], per epoch
// parity.  n8 (16-B vectors) must split evenly: n8 % world == 0.
__global__ __launch_bounds__(256) void car_twoshot_kernel(CarArgs a) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  unsigned* my_sig = reinterpret_cast<unsigned*>(a.sig[a.rank]);
  const unsigned epoch = car_epoch(my_sig, tid);
  const long par = (long)(epoch & 1) * a.half_elems;
  const long slice8 = a.n8 / a.world;                       // vectors per slice
  const long sub = (slice8 + nb - 1) / nb;                  // per block
  const long lo = (long)b * sub, hi = min(slice8, lo + sub);  // this block's sub-range of a slice
  const long res_off = a.n8 * 8;                            // reduced-slice region (elements)
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
  // 1. every slice's sub-range b of the input -> own buffer
  uint4* mine = reinterpret_cast<uint4*>(reinterpret_cast<unsigned short*>(a.data[a.rank]) + par);
  const uint4* in = reinterpret_cast<const uint4*>(a.inp);
  for (int sl = 0; sl < a.world; ++sl)
    for (long i = lo + tid; i < hi; i += 256) mine[sl * slice8 + i] = in[sl * slice8 + i];
  __threadfence_system();
  __syncthreads();
  car_signal_wait(a, my_sig, b, tid, epoch, 0);
  // 2. reduce this rank's slice, sub-range b, over all ranks -> own reduced region
  unsigned short* red = reinterpret_cast<unsigned short*>(a.data[a.rank]) + par + res_off;
  for (long i = lo + tid; i < hi; i += 256) {
    float acc[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] = 0.f;
    for (int r = 0; r < a.world; ++r) {
      const u32x4* src = reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned short*>(a.data[r]) + par);
      const u32x4 v = __builtin_nontemporal_load(src + (long)a.rank * slice8 + i);
      const unsigned short* h = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += bf2f(h[j]);
    }
    store8(red + i * 8, acc);
  }
  __threadfence_system();
  __syncthreads();
  car_signal_wait(a, my_sig, b, tid, epoch, 1);
  // 3. gather every rank's reduced slice, sub-range b
  for (int sl = 0; sl < a.world; ++sl) {
    const u32x4* src =
        reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned short*>(a.data[sl]) + par + res_off);
    u32x4* dst = reinterpret_cast<u32x4*>(a.out) + (long)sl * slice8;
    for (long i = lo + tid; i < hi; i += 256) dst[i] = __builtin_nontemporal_load(src + i);
  }
  car_finish(my_sig, nb, tid, epoch);
}

// Row-parallel projection partials -> all-reduce + bias + residual add + RMSNorm in ONE kernel
// (TP decode: the o / down projections' partial sums are reduced and the next sub-layer's input
// norm applied without the RCCL / one-shot all-reduce output round-tripping through HBM and a
// separate add+norm launch).  Block b owns rows b, b + nb, ...: it stages them in its own
// buffer, exchanges one flag per peer (the same rows on every rank), then for each row
//   o = bf16(sum_r part_r + bias); s = bf16(o + res) -> res_out; y = bf16(s * rsqrt(mean(s^2) + eps) * w)
// exactly as the unfused all-reduce -> add_rmsnorm (and decode_fin_add_rmsnorm) round.
struct CarNormArgs {
  const unsigned short* bias;  // [N] or nullptr
  const unsigned short* res;   // [M, N]
  const unsigned short* nw;    // [N]
  unsigned short* res_out;     // [M, N]
  int M, N;
  float eps;
};

__global__ __launch_bounds__(256) void car_add_rmsnorm_kernel(CarArgs a, CarNormArgs c) {
  extern __shared__ __attribute__((aligned(16))) float srow[];
  __shared__ float red[4];
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  unsigned* my_sig = reinterpret_cast<unsigned*>(a.sig[a.rank]);
  const unsigned epoch = car_epoch(my_sig, tid);
  const long par = (long)(epoch & 1) * a.half_elems;
  const int N = c.N, n8 = N / 8;
  unsigned short* mine = reinterpret_cast<unsigned short*>(a.data[a.rank]) + par;
  for (int m = b; m < c.M; m += nb)
    for (int i = tid; i < n8; i += 256)
      reinterpret_cast<uint4*>(mine + (long)m * N)[i] = reinterpret_cast<const uint4*>(a.inp + (long)m * N)[i];
  __threadfence_system();
  __syncthreads();
  car_signal_wait(a, my_sig, b, tid, epoch);
  using u32x4 = __attribute__((ext_vector_type(4))) unsigned int;
  for (int m = b; m < c.M; m += nb) {
    const long base = (long)m * N;
    float ss = 0.f;
    for (int i = tid; i < n8; i += 256) {
      float acc[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = 0.f;
      for (int r = 0; r < a.world; ++r) {
        const u32x4* src = reinterpret_cast<const u32x4*>(reinterpret_cast<const unsigned short*>(a.data[r]) + par + base);
        const u32x4 v = __builtin_nontemporal_load(src + i);
        const unsigned short* h = reinterpret_cast<const unsigned short*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(h[j]);
      }
      float rv[8], bv[8];
      load8(c.res + base + i * 8, rv);
      if (c.bias) load8(c.bias + i * 8, bv);
      float sv[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float o = bf2f(f2bf(acc[j]));
        if (c.bias) o = bf2f(f2bf(o + bv[j]));
        sv[j] = bf2f(f2bf(o + rv[j]));
        srow[i * 8 + j] = sv[j];
        ss += sv[j] * sv[j];
      }
      store8(c.res_out + base + i * 8, sv);
    }
    // block sum of ss (4 waves)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
    if ((tid & 63) == 0) red[tid >> 6] = ss;
    __syncthreads();
    const float rs = rsqrtf((red[0] + red[1] + red[2] + red[3]) / (float)N + c.eps);
    for (int i = tid; i < n8; i += 256) {
      float wv[8], yv[8];
      load8(c.nw + i * 8, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) yv[j] = srow[i * 8 + j] * rs * wv[j];
      store8(a.out + base + i * 8, yv);
    }
    __syncthreads();  // srow / red reused by the block's next row
  }
  car_finish(my_sig, nb, tid, epoch);
}

}  // namespace

int64_t car_malloc(int64_t bytes) {
  void* p = nullptr;
  LLMCTL_HIP_CHECK(hipExtMallocWithFlags(&p, (size_t)bytes, hipDeviceMallocUncached));
  LLMCTL_HIP_CHECK(hipMemset(p, 0, (size_t)bytes));
  LLMCTL_HIP_CHECK(hipDeviceSynchronize());
  return reinterpret_cast<int64_t>(p);
}

void car_free(int64_t ptr) { LLMCTL_HIP_CHECK(hipFree(reinterpret_cast<void*>(ptr))); }

at::Tensor car_ipc_handle(int64_t ptr) {
  hipIpcMemHandle_t h;
  LLMCTL_HIP_CHECK(hipIpcGetMemHandle(&h, reinterpret_cast<void*>(ptr)));
  auto t = at::empty({(long)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(t.data_ptr(), &h, sizeof(h));
  return t;
}

int64_t car_ipc_open(const at::Tensor& handle) {
  LLMCTL_CHECK(handle.numel() == (long)sizeof(hipIpcMemHandle_t) && handle.device().is_cpu(), "car_ipc_open: handle");
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  void* p = nullptr;
  LLMCTL_HIP_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  return reinterpret_cast<int64_t>(p);
}

void car_ipc_close(int64_t ptr) { LLMCTL_HIP_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr))); }

int64_t car_sig_words() { return CAR_SIG_WORDS; }

// error word of this rank's signal buffer (host read; 0 = ok)
int64_t car_error(int64_t sig_ptr) {
  unsigned v = 0;
  LLMCTL_HIP_CHECK(hipMemcpy(&v, reinterpret_cast<unsigned*>(sig_ptr) + CAR_ERROR, 4, hipMemcpyDeviceToHost));
  return v;
}

void car_allreduce(const at::Tensor& inp, at::Tensor& out, const at::Tensor& data_ptrs, const at::Tensor& sig_ptrs,
                   int64_t rank, int64_t world, int64_t half_bytes) {
  LLMCTL_CHECK(inp.is_cuda() && inp.is_contiguous() && out.is_contiguous() && inp.scalar_type() == at::kBFloat16 &&
                   out.scalar_type() == at::kBFloat16 && out.numel() == inp.numel(),
               "car_allreduce: contiguous bf16 in/out of equal size");
  LLMCTL_CHECK(world >= 1 && world <= CAR_MAX_RANKS && rank >= 0 && rank < world, "car_allreduce: world <= 8");
  LLMCTL_CHECK(inp.numel() % 8 == 0 && inp.numel() * 2 <= half_bytes, "car_allreduce: numel % 8 and size <= buffer");
  LLMCTL_CHECK(data_ptrs.device().is_cpu() && sig_ptrs.device().is_cpu() && data_ptrs.numel() == world &&
                   sig_ptrs.numel() == world && data_ptrs.scalar_type() == at::kLong,
               "car_allreduce: CPU int64 pointer tables");
  const c10::DeviceGuard g(inp.device());
  CarArgs a{};
  a.inp = bf_ptr(inp);
  a.out = bf_mut(out);
  for (int r = 0; r < world; ++r) {
    a.data[r] = (unsigned long long)data_ptrs.data_ptr<int64_t>()[r];
    a.sig[r] = (unsigned long long)sig_ptrs.data_ptr<int64_t>()[r];
  }
  a.rank = (int)rank;
  a.world = (int)world;
  a.n8 = inp.numel() / 8;
  a.half_elems = half_bytes / 2;
  const int nb = (int)std::max<long>(1, std::min<long>(CAR_MAX_BLOCKS, (a.n8 + 255) / 256));
  hipLaunchKernelGGL(car_oneshot_kernel, dim3(nb), dim3(256), 0, stream(), a);
}

// two-shot variant: the buffer half must hold the input copy AND the reduced slice
void car_allreduce_twoshot(const at::Tensor& inp, at::Tensor& out, const at::Tensor& data_ptrs,
                           const at::Tensor& sig_ptrs, int64_t rank, int64_t world, int64_t half_bytes) {
  LLMCTL_CHECK(inp.is_cuda() && inp.is_contiguous() && out.is_contiguous() && inp.scalar_type() == at::kBFloat16 &&
                   out.scalar_type() == at::kBFloat16 && out.numel() == inp.numel(),
               "car_allreduce_twoshot: contiguous bf16 in/out of equal size");
  LLMCTL_CHECK(world >= 1 && world <= CAR_MAX_RANKS && rank >= 0 && rank < world, "car_allreduce_twoshot: world <= 8");
  LLMCTL_CHECK(inp.numel() % (8 * world) == 0 && inp.numel() * 2 + inp.numel() * 2 / world <= half_bytes,
               "car_allreduce_twoshot: numel % (8 world) and input + slice <= buffer half");
  LLMCTL_CHECK(data_ptrs.device().is_cpu() && sig_ptrs.device().is_cpu() && data_ptrs.numel() == world &&
                   sig_ptrs.numel() == world && data_ptrs.scalar_type() == at::kLong,
               "car_allreduce_twoshot: CPU int64 pointer tables");
  const c10::DeviceGuard g(inp.device());
  CarArgs a{};
  a.inp = bf_ptr(inp);
  a.out = bf_mut(out);
  for (int r = 0; r < world; ++r) {
    a.data[r] = (unsigned long long)data_ptrs.data_ptr<int64_t>()[r];
    a.sig[r] = (unsigned long long)sig_ptrs.data_ptr<int64_t>()[r];
  }
  a.rank = (int)rank;
  a.world = (int)world;
  a.n8 = inp.numel() / 8;
  a.half_elems = half_bytes / 2;
  const long slice8 = a.n8 / world;
  const int nb = (int)std::max<long>(1, std::min<long>(CAR_MAX_BLOCKS, (slice8 + 255) / 256));
  hipLaunchKernelGGL(car_twoshot_kernel, dim3(nb), dim3(256), 0, stream(), a);
}

// partial [M, N] (this rank's row-parallel projection output) -> (y = rmsnorm(res + sum + bias) * w, res_out)
std::tuple<at::Tensor, at::Tensor> car_allreduce_add_rmsnorm(const at::Tensor& partial, const c10::optional<at::Tensor>& bias,
                                                             const at::Tensor& res, const at::Tensor& nw, double eps,
                                                             const at::Tensor& data_ptrs, const at::Tensor& sig_ptrs,
                                                             int64_t rank, int64_t world, int64_t half_bytes) {
  LLMCTL_CHECK(partial.is_cuda() && partial.is_contiguous() && partial.scalar_type() == at::kBFloat16 &&
                   partial.dim() == 2 && res.sizes() == partial.sizes() && res.is_contiguous() &&
                   res.scalar_type() == at::kBFloat16,
               "car_allreduce_add_rmsnorm: contiguous bf16 partial / residual [M, N]");
  const long M = partial.size(0), N = partial.size(1);
  LLMCTL_CHECK(nw.is_contiguous() && nw.numel() == N && nw.scalar_type() == at::kBFloat16,
               "car_allreduce_add_rmsnorm: norm weight bf16 [N]");
  const bool has_b = bias.has_value() && bias->defined();
  if (has_b) {
    LLMCTL_CHECK(bias->is_contiguous() && bias->numel() == N && bias->scalar_type() == at::kBFloat16,
                 "car_allreduce_add_rmsnorm: bias bf16 [N]");
  }
  LLMCTL_CHECK(N % 8 == 0 && N <= 16384 && M * N * 2 <= half_bytes, "car_allreduce_add_rmsnorm: N % 8, N <= 16384, fits");
  LLMCTL_CHECK(world >= 1 && world <= CAR_MAX_RANKS && rank >= 0 && rank < world, "car_allreduce_add_rmsnorm: world <= 8");
  LLMCTL_CHECK(data_ptrs.device().is_cpu() && sig_ptrs.device().is_cpu() && data_ptrs.numel() == world &&
                   sig_ptrs.numel() == world && data_ptrs.scalar_type() == at::kLong,
               "car_allreduce_add_rmsnorm: CPU int64 pointer tables");
  const c10::DeviceGuard g(partial.device());
  auto y = at::empty_like(partial);
  auto res_out = at::empty_like(partial);
  CarArgs a{};
  a.inp = bf_ptr(partial);
  a.out = bf_mut(y);
  for (int r = 0; r < world; ++r) {
    a.data[r] = (unsigned long long)data_ptrs.data_ptr<int64_t>()[r];
    a.sig[r] = (unsigned long long)sig_ptrs.data_ptr<int64_t>()[r];
  }
  a.rank = (int)rank;
  a.world = (int)world;
  a.n8 = M * N / 8;
  a.half_elems = half_bytes / 2;
  CarNormArgs c{has_b ? bf_ptr(*bias) : nullptr, bf_ptr(res), bf_ptr(nw), bf_mut(res_out), (int)M, (int)N, (float)eps};
  const int nb = (int)std::max<long>(1, std::min<long>(CAR_MAX_BLOCKS, M));
  hipLaunchKernelGGL(car_add_rmsnorm_kernel, dim3(nb), dim3(256), (size_t)N * 4, stream(), a, c);
  return {y, res_out};
}

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) {
  m.impl("car_allreduce", &car_allreduce);
  m.impl("car_allreduce_twoshot", &car_allreduce_twoshot);
  m.impl("car_allreduce_add_rmsnorm", &car_allreduce_add_rmsnorm);
}
// the tensor-less buffer/IPC helpers are registered as catch-all kernels in bindings.cpp

}  // namespace llmctl
