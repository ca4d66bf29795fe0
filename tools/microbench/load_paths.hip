// Per-CU global->LDS / global->VGPR load throughput on MI355X (L2-resident source).
// Build: hipcc --offload-arch=gfx950 -O3 load_paths.hip -o load_paths
// Each workgroup (NW waves) streams ITERS x 64 KB from a 4 MB (L2-resident per XCD) buffer.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef int i32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ i32x4 rsrc(const void* base) {
  unsigned long a = (unsigned long)base;
  i32x4 r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = -1;
  r[3] = 0x00020000;
  return r;
}

// MODE 0: global_load_lds_dwordx4 (flat 64-bit addr); 1: buffer_load_dwordx4 ... lds;
// 2: global_load_dwordx4 -> VGPR (sum kept live); 3: global_load_dwordx4 -> ds_write_b128
template <int MODE>
__global__ void k(const unsigned short* __restrict__ src, float* out, int iters, int span_kb) {
  __shared__ __attribute__((aligned(1024))) unsigned char smem[65536];
  const int tid = threadIdx.x, nthr = blockDim.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const unsigned lds0 = __builtin_amdgcn_readfirstlane((unsigned)(uintptr_t)(__attribute__((address_space(3))) unsigned char*)smem);
  const long span = (long)span_kb * 1024 / 2;  // elements
  const long base = ((long)blockIdx.x * 65536 / 2) % span;
  i32x4 rs = rsrc(src);
  uint4 accv = make_uint4(0, 0, 0, 0);
  const int per = 65536 / (nthr * 16);  // 16-B pieces per thread per 64 KB tile
  for (int it = 0; it < iters; ++it) {
    const long off = (base + (long)it * 32768) % span;
    for (int p = 0; p < per; ++p) {
      const long e = off + ((long)p * nthr + tid) * 8;
      const unsigned l = lds0 + (p * nthr + wave * 64) * 16;
      if constexpr (MODE == 0) {
        asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(src + (e % span)), "s"(l) : "memory");
      } else if constexpr (MODE == 1) {
        unsigned vo = (unsigned)((e % span) * 2);
        asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(vo), "s"(rs), "s"(l) : "memory");
      } else if constexpr (MODE == 2) {
        uint4 v = *reinterpret_cast<const uint4*>(src + (e % span));
        accv.x ^= v.x; accv.y ^= v.y; accv.z ^= v.z; accv.w ^= v.w;
      } else {
        uint4 v = *reinterpret_cast<const uint4*>(src + (e % span));
        *reinterpret_cast<uint4*>(smem + (p * nthr + tid) * 16) = v;
      }
    }
    if constexpr (MODE <= 1) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  out[blockIdx.x * nthr + tid] = ((float*)smem)[tid] + (float)(accv.x ^ accv.y ^ accv.z ^ accv.w);
}

int main() {
  const long bytes = 64L << 20;
  unsigned short* src;
  float* out;
  hipMalloc(&src, bytes);
  hipMemset(src, 1, bytes);
  hipMalloc(&out, 256 * 1024 * 4 * 4);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int iters = 2000;
  for (int span_kb : {2048, 65536}) {
    for (int nthr : {256, 512}) {
      for (int mode = 0; mode < 4; ++mode) {
        for (int rep = 0; rep < 2; ++rep) {
          hipEventRecord(a);
          switch (mode) {
            case 0: hipLaunchKernelGGL(k<0>, dim3(256), dim3(nthr), 0, 0, src, out, iters, span_kb); break;
            case 1: hipLaunchKernelGGL(k<1>, dim3(256), dim3(nthr), 0, 0, src, out, iters, span_kb); break;
            case 2: hipLaunchKernelGGL(k<2>, dim3(256), dim3(nthr), 0, 0, src, out, iters, span_kb); break;
            default: hipLaunchKernelGGL(k<3>, dim3(256), dim3(nthr), 0, 0, src, out, iters, span_kb); break;
          }
          hipEventRecord(b);
          hipEventSynchronize(b);
          float ms;
          hipEventElapsedTime(&ms, a, b);
          if (rep == 1) {
            double tb = 256.0 * iters * 65536 / (ms * 1e-3) / 1e12;
            printf("span %6d KB  threads %d  mode %d  %.3f ms  %.2f TB/s  %.1f B/clk/CU@2.1GHz\n", span_kb, nthr, mode, ms,
                   tb, tb * 1e12 / 256 / 2.1e9);
          }
        }
      }
    }
  }
  return 0;
}
