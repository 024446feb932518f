// LDS access helpers shared by the fused QKV + attention kernels (qkv_attn.hip, qkv_attn_ws.hip).
//
// The attention reads go through inline asm and are waited for with counted lgkmcnt waits:
// for compiler-visible LDS loads the waitcnt pass (a) put one lgkmcnt(0) after a whole batch
// of reads instead of counted waits, and (b) drained the LDS-DMA stream in flight into other
// LDS buffers (vmcnt(0)) before the first read, since it cannot tell the DMA destination apart.
#pragma once
#include "atpu/common.h"

namespace atpu {

// operand-image swizzle (128-B rows, 16-B chunk c of row r at slot c ^ ((r >> 1) & 7))
__device__ __forceinline__ int hsw(int r, int c) { return c ^ ((r >> 1) & 7); }

// attention-image swizzle: per sequence, Q, K, V of a head as [128][128 B] bf16 images, 16-B
// chunk c of row r at slot c ^ (r & 7). One swizzle is bank-conflict-free for the 16-B image
// writes (8-lane groups = 8 consecutive rows of one chunk, mod 32 banks), the ds_read_b128
// fragment reads of Q and K, and the transposed ds_read_b64_tr_b16 reads of V (32-lane groups
// = 8 rows x 2 chunks, mod 64 banks) (tools/lds_banks_qkv_attn.py)
constexpr int kAttnImg = 128 * 128;
__device__ __forceinline__ int asw(int r, int c) { return c ^ (r & 7); }

// v_permlane16_swap: lane rows (16-lane groups) 1 and 3 of x trade places with rows 0 and 2
// of y. On the two packed halves of MFMA fragments of row blocks i (x) and i+1 (y) it leaves
// lane row G holding 8 consecutive columns (G >> 1: which 8 of the 16) of block i + (G & 1):
// one 16-B LDS write per lane instead of two 8-B writes. The s_nop covers the VALU-write ->
// permlane-read hazard.
__device__ __forceinline__ void swap16(unsigned& x, unsigned& y) {
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
}

__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}

__device__ __forceinline__ bf16x8 ds_read128(const char* p) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(lds_addr(p)));
  return r;
}
__device__ __forceinline__ u32x4 ds_read128u(const char* p) {
  u32x4 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(lds_addr(p)));
  return r;
}
__device__ __forceinline__ void ds_write128(char* p, u32x4 v) {
  asm volatile("ds_write_b128 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}

// s_waitcnt lgkmcnt(N) that the two registers it retires pass through (so their consumers
// cannot be scheduled above it)
template <int N>
__device__ __forceinline__ void lgkm_wait(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
}

typedef short hv4s __attribute__((vector_size(8)));
// ds_read_b64_tr_b16 (per 16-lane group: lane 4q+p addresses row q, elements 4p..4p+3 of a
// 4 x 16 block; lane i receives column i of the 4 rows)
__device__ __forceinline__ bf16x4 tr16(const char* p) {
  hv4s r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(lds_addr(p)));
  return __builtin_bit_cast(bf16x4, r);
}

}  // namespace atpu
