// L2 prefetch of the next decode kernel's weight rows by one extra wave of the current
// kernel (gemm_bf16.hip decode GEMV, decode.hip split cross attention).
//
// The wave issues a dword load per 128-B line of the rows that the NEXT kernel's workgroups
// b' = bid + k * nblk will read (`rpb` rows each), waits for them and exits; the compute waves
// never wait for it. Workgroups are dealt to the XCDs round robin by linear id, so with
// nblk % 8 == 0 the lines land in the L2 of the XCD whose workgroup reads them next (a
// speed-only assumption: another placement only loses the L2 hit). The loads are 4-byte
// LDS-DMAs into a scratch nobody reads: a VGPR-destination load issued from inline asm
// would let the compiler reuse its register before the data returns.
#pragma once

#include "atpu/common.h"

namespace atpu {

struct L2Pf {
  const bf16* w;
  int ld, k, n, rpb;  // rpb: weight rows per workgroup of the next kernel (16, or 32 for RowStats)
};

// BARRIERS: raw s_barriers to take (the workgroup's barriers the compute waves pass), issued
// with the loads still in flight (__syncthreads would drain them first and hold the compute
// waves), then the drain before the wave ends
template <int BARRIERS>
__device__ __forceinline__ void l2_prefetch_rows(const L2Pf& pf, int lane, char* scratch, int bid, int nblk) {
  const int lpr = (pf.k * 2 + 127) / 128;  // 128-B lines per row
  const int blocks = (pf.n + pf.rpb - 1) / pf.rpb;
  // fewer next blocks than workgroups here (e.g. 32 RowStats slabs of an 8 MB weight behind 256
  // workgroups): the `share` workgroups bid = bb (mod blocks) -- the same XCD as block bb when
  // blocks % 8 == 0 -- split block bb's lines, instead of 32 waves streaming 256 KB each while
  // the kernel waits for them to end
  const int share = (blocks < nblk && nblk % blocks == 0) ? nblk / blocks : 1;
  for (int bb = (share > 1 ? bid % blocks : bid); bb < blocks; bb += (share > 1 ? blocks : nblk)) {
    const int r0 = bb * pf.rpb, nl = min(pf.rpb, pf.n - r0) * lpr;
    const int part = share > 1 ? bid / blocks : 0;
    const int l0 = (int)((long)nl * part / share), l1 = (int)((long)nl * (part + 1) / share);
    for (int i0 = l0; i0 < l1; i0 += 64) {  // wave-uniform trip count: every lane issues the DMA
      const int i = min(i0 + lane, l1 - 1);
      const int r = r0 + i / lpr, l = i - (i / lpr) * lpr;
      const char* p = reinterpret_cast<const char*>(pf.w + (size_t)r * pf.ld) + l * 128;
      __builtin_amdgcn_global_load_lds((const ATPU_GLOBAL_AS void*)p, (ATPU_LDS_AS void*)scratch, 4, 0, 0);
    }
    if (share > 1) break;  // one block per workgroup
  }
#pragma unroll
  for (int b = 0; b < BARRIERS; ++b) asm volatile("s_barrier" ::: "memory");
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

}  // namespace atpu
