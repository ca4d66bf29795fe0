// Shared pieces of the flash-attention kernels (gfx950, MFMA 32x32x16 bf16).
//
// MFMA fragment maps used throughout (CDNA guide §3):
//   A (32x16): lane l (r=l&31, h=l>>5) holds A[r][8h+j], j=0..7
//   B (16x32): lane l holds B[8h+j][r]
//   C/D (32x32, 16 regs): reg i of lane l is C[row=(i&3)+8(i>>2)+4h][col=r]
// "Swapped" products keep the key index on the MFMA *row* (registers) and the query on the
// lane, so softmax rows are lane-local and the probability tile P^T feeds the next MFMA as
// its B operand with no lane movement (guide §3, accumulator-as-operand).
#pragma once
#include "common.h"

namespace llmctl {
namespace attn {

using bf16x8_t = __attribute__((ext_vector_type(8))) __bf16;
using s4_t = __attribute__((ext_vector_type(4))) short;
using s8_t = __attribute__((ext_vector_type(8))) short;
using f32x16 = __attribute__((ext_vector_type(16))) float;
using lds_s4 = __attribute__((address_space(3))) s4_t;

__device__ __forceinline__ f32x16 mfma32(bf16x8_t a, bf16x8_t b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// x combined with lane l^32's x in one v_permlane32_swap (no LDS round trip, unlike __shfl_xor)
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_add(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}

// row index of register i of a 32x32 accumulator for lane half h
__device__ __forceinline__ int acc_row(int i, int h) { return (i & 3) + 8 * (i >> 2) + 4 * h; }

// ---- LDS tile images ----------------------------------------------------------------------
// Tiles are [rows][HD] bf16, rows of HD*2 bytes, addressed in 16-byte chunks (8 bf16).
//   "row image"  (read by ds_read_b128, lanes = different rows, same chunk):
//        chunk' = chunk ^ swz_row(row)
//   "tr image"   (read by ds_read_b64_tr_b16, 4 rows x 64 B per 32-lane half):
//        chunk' = chunk ^ swz_tr(row)
template <int HD>
__device__ __forceinline__ int swz_row(int row) {
  if constexpr (HD == 128) return row & 15;       // 256-B rows: 16 rows -> 16 distinct chunks
  else return (row >> 1) & 7;                     // 128-B rows: 2 rows per 256-B bank row
}
template <int HD>
__device__ __forceinline__ int swz_tr(int row) {
  if constexpr (HD == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
}

template <int HD>
__device__ __forceinline__ int row_off(int row, int chunk) {  // byte offset, row image
  return row * (HD * 2) + ((chunk ^ swz_row<HD>(row)) << 4);
}
template <int HD>
__device__ __forceinline__ int tr_off(int row, int chunk) {  // byte offset, tr image
  return row * (HD * 2) + ((chunk ^ swz_tr<HD>(row)) << 4);
}

__device__ __forceinline__ bf16x8_t lds_read_b128(const unsigned char* base, int off) {
  return *reinterpret_cast<const bf16x8_t*>(base + off);
}

// A-operand fragment of X^T where X [rows][HD] is stored as a tr image: lane gets
// X[row0 + 4h + j][col0 + r] for j<4 and X[row0 + 8 + 4h + (j-4)][col0 + r] for j>=4,
// i.e. the 32x16 A tile "X^T[col0..col0+31][row0..row0+15]" in the k-permuted order that
// matches an accumulator-as-B operand (reg block 8s..8s+7).
template <int HD>
__device__ __forceinline__ bf16x8_t tr_frag(const unsigned char* base, int row0, int col0, int lane) {
  const int h = lane >> 5;
  const int i16 = lane & 15;
  const int q = i16 >> 2, p = i16 & 3;
  const int col = col0 + 16 * ((lane >> 4) & 1) + 4 * p;
  const int chunk = col >> 3;
  const int sub = (col & 7) * 2;  // 0 or 8 bytes
  const int r1 = row0 + 4 * h + q;
  const int r2 = r1 + 8;
  s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + tr_off<HD>(r1, chunk) + sub));
  s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + tr_off<HD>(r2, chunk) + sub));
  s8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// tr_frag with the lane's byte offsets precomputed (tr_frag_offs): for row0 % 16 == 0 the tr-image
// swizzle of rows row0 + 4h + q (+ 8) depends on the lane only, so the address of every fragment
// of a tile is base + row0 * 2 HD + the lane's (lo, hi) offset of its 32-column block — the row /
// slot part folds into the ds_read immediate (no per-read address VALU in the loop)
template <int HD>
__device__ __forceinline__ void tr_frag_offs(int col0, int lane, int& lo, int& hi) {
  const int h = lane >> 5;
  const int i16 = lane & 15;
  const int q = i16 >> 2, p = i16 & 3;
  const int col = col0 + 16 * ((lane >> 4) & 1) + 4 * p;
  const int chunk = col >> 3;
  const int sub = (col & 7) * 2;
  lo = tr_off<HD>(4 * h + q, chunk) + sub;
  hi = tr_off<HD>(8 + 4 * h + q, chunk) + sub;
}
template <int HD>
__device__ __forceinline__ bf16x8_t tr_frag_at(const unsigned char* base, int row0, int lo, int hi) {
  s4_t a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + row0 * (HD * 2) + lo));
  s4_t b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + row0 * (HD * 2) + hi));
  s8_t v = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

// natural-order A fragment of X^T (k = 8h + j) from a tr image: X[row0 + 8h + j][col0 + r]
template <int HD>
__device__ __forceinline__ bf16x8_t tr_frag_nat(const unsigned char* base, int row0, int col0, int lane) {
  const int h = lane >> 5;
  const int i16 = lane & 15;
  const int q = i16 >> 2, p = i16 & 3;
  const int col = col0 + 16 * ((lane >> 4) & 1) + 4 * p;
  const int chunk = col >> 3;
  const int sub = (col & 7) * 2;
  const int r1 = row0 + 8 * h + q;
  const int r2 = r1 + 4;
  s4_t lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + tr_off<HD>(r1, chunk) + sub));
  s4_t hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4*)(base + tr_off<HD>(r2, chunk) + sub));
  s8_t v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
  return __builtin_bit_cast(bf16x8_t, v);
}

__device__ __forceinline__ bf16x8_t to_bf16x8(const float* x) {
  bf16x8_t v;
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = (__bf16)x[j];
  return v;
}

__device__ __forceinline__ uint4 gload16(const unsigned short* p) { return *reinterpret_cast<const uint4*>(p); }

// ---- LDS DMA (global_load_lds) ---------------------------------------------------------------
// One wave-instruction writes 64 lanes x {16, 4} B to LDS bytes [lds_byte, +1024 / +256),
// lane-linear; the global source address is per lane (a swizzled image is built by permuting
// the SOURCE, guide §5.4 rule 21).  Inline asm: through the builtin, hipcc drains vmcnt(0)
// before every later ds_read; here ordering is explicit (counted vmcnt + s_barrier).
__device__ __forceinline__ void dma16(const void* g, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(g), "s"(lds_byte) : "memory");
}
__device__ __forceinline__ void dma4(const void* g, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dword %0, off" ::"v"(g), "s"(lds_byte) : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait() {
  static_assert(N >= 0 && N <= 15, "vmcnt immediate");
  if constexpr (N == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  else if constexpr (N == 5) asm volatile("s_waitcnt vmcnt(5)" ::: "memory");
  else if constexpr (N == 9) asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  else static_assert(N == 0 || N == 5 || N == 9, "add the immediate");
}
// Buffer-resource LDS-DMA (buffer_load_dwordx4 ... lds): base and record count are scalar, so a
// per-tile move of the source window costs SALU only; loads at offsets >= num_records return 0.
using i32x4_t = __attribute__((ext_vector_type(4))) int;
__device__ __forceinline__ i32x4_t buf_rsrc(const void* base, unsigned num_records) {
  const unsigned long a = (unsigned long)base;
  i32x4_t r;
  r[0] = __builtin_amdgcn_readfirstlane((int)(a & 0xffffffffu));
  r[1] = __builtin_amdgcn_readfirstlane((int)((a >> 32) & 0xffff));
  r[2] = __builtin_amdgcn_readfirstlane((int)num_records);
  r[3] = 0x00020000;  // raw buffer, 32-bit data format
  return r;
}
__device__ __forceinline__ void buf_dma16(i32x4_t rsrc, unsigned voff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(lds_byte)
               : "memory");
}
__device__ __forceinline__ void buf_dma4(i32x4_t rsrc, unsigned voff, unsigned lds_byte) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dword %0, %1, 0 offen lds" ::"v"(voff), "s"(rsrc),
               "s"(lds_byte)
               : "memory");
}
template <int N>
__device__ __forceinline__ void vm_wait_n() {
  static_assert(N >= 0 && N <= 63, "vmcnt immediate");
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N) : "memory");
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return __builtin_amdgcn_readfirstlane(
      (unsigned)(uintptr_t)(const __attribute__((address_space(3))) unsigned char*)p);
}

}  // namespace attn
}  // namespace llmctl
