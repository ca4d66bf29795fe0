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
// signal buffer layout (uint32): flags[CAR_MAX_BLOCKS][CAR_MAX_RANKS], then epoch, done, error
constexpr int CAR_EPOCH = CAR_MAX_BLOCKS * CAR_MAX_RANKS;
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

__global__ __launch_bounds__(256) void car_oneshot_kernel(CarArgs a) {
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  unsigned* my_sig = reinterpret_cast<unsigned*>(a.sig[a.rank]);
  __shared__ unsigned s_epoch;
  if (tid == 0) s_epoch = __hip_atomic_load(my_sig + CAR_EPOCH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1;
  __syncthreads();
  const unsigned epoch = s_epoch;
  const long par = (long)(epoch & 1) * a.half_elems;
  // 1. input slice -> own buffer
  uint4* mine = reinterpret_cast<uint4*>(reinterpret_cast<unsigned short*>(a.data[a.rank]) + par);
  const uint4* in = reinterpret_cast<const uint4*>(a.inp);
  for (long i = (long)b * 256 + tid; i < a.n8; i += (long)nb * 256) mine[i] = in[i];
  __threadfence_system();
  __syncthreads();
  // 2. signal every peer, then wait for every peer's signal for this block
  if (tid < a.world) {
    unsigned* peer = reinterpret_cast<unsigned*>(a.sig[tid]);
    __hip_atomic_store(peer + b * CAR_MAX_RANKS + a.rank, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    unsigned* f = my_sig + b * CAR_MAX_RANKS + tid;
    long spins = 0;
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      __builtin_amdgcn_s_sleep(2);
      if (++spins > (1L << 26)) {  // ~seconds: a peer is gone; report instead of hanging
        __hip_atomic_store(my_sig + CAR_ERROR, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        break;
      }
    }
  }
  __syncthreads();
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
  // 4. last block to finish advances the epoch (device-side: graph replays stay correct)
  __syncthreads();
  if (tid == 0) {
    const unsigned d = __hip_atomic_fetch_add(my_sig + CAR_DONE, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (d == (unsigned)nb - 1) {
      __hip_atomic_store(my_sig + CAR_DONE, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(my_sig + CAR_EPOCH, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
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

TORCH_LIBRARY_IMPL(llmctl, CUDA, m) { m.impl("car_allreduce", &car_allreduce); }
// the tensor-less buffer/IPC helpers are registered as catch-all kernels in bindings.cpp

}  // namespace llmctl
