// Batched GPU tokenizer: packed UTF-8 rows -> BERT ids.
//
// Spec ("atpu-hash-wordpiece v1", CPU twin: agent_tpu_amd/tokenizer.py):
//   bytes 0x09-0x0D, 0x20            separator
//   other bytes < 0x20, 0x7F         separator (control, dropped)
//   ASCII punctuation                one single-byte token each
//   everything else (alnum, >=0x80)  word bytes, ASCII A-Z lower-cased
//   a word is cut into pieces of <= 24 bytes; piece 0 is FNV-1a-32 hashed from
//   the standard basis, later pieces from the FNV state of "##" (WordPiece's
//   continuation marker); id = 1000 + hash % (vocab - 1000).
//   ids = [CLS=101] + first S-2 tokens + [SEP=102] + [PAD=0]...; len = n + 2.
//
// One 64-wide wave per row. The row is staged into LDS, then scanned 64 bytes
// per step: each lane classifies its byte (and the byte 64 further on), token
// starts are found against the left neighbour (shfl_up; chunk-carry through lane
// 63), a word's length is the run of word bytes from its start in the 128-bit
// ballot of the two chunks (one ctz; words of 64+ bytes fall back to a walk), and
// an inclusive wave scan of piece counts gives every token its output slot. The
// lane at a token start hashes its piece from 7 aligned dwords of LDS realigned
// with v_alignbyte (no dependent byte loads; the byte loop runs to the longest
// piece of the step). The scan stops as soon as S-2 tokens exist, so long rows
// cost only the bytes that are used. (The byte-walking form spent ~90 us on a
// 1024-row batch, latency-bound on dependent LDS reads.)
#include "atpu/common.h"
#include "atpu/kernels.h"

namespace atpu {
namespace {

constexpr int kMaxRowBytes = 4096;
constexpr int kPiece = 24;
constexpr uint32_t kFnvBasis = 2166136261u;
constexpr uint32_t kFnvPrime = 16777619u;

__device__ __forceinline__ int byte_class(uint32_t c) {
  if (c == 0x20 || (c >= 0x09 && c <= 0x0D)) return 0;
  if (c < 0x20 || c == 0x7F) return 0;
  if ((c >= 0x21 && c <= 0x2F) || (c >= 0x3A && c <= 0x40) || (c >= 0x5B && c <= 0x60) || (c >= 0x7B && c <= 0x7E))
    return 1;
  return 2;
}

__device__ __forceinline__ uint32_t fnv_step(uint32_t h, uint32_t c) {
  if (c >= 'A' && c <= 'Z') c += 32;
  return (h ^ c) * kFnvPrime;
}

__device__ __forceinline__ int wave_inclusive_scan(int v, int lane) {
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int t = __shfl_up(v, o, 64);
    if (lane >= o) v += t;
  }
  return v;
}

__global__ __launch_bounds__(256) void tokenize_kernel(const uint8_t* __restrict__ text,
                                                       const int32_t* __restrict__ offsets, int32_t* __restrict__ ids,
                                                       int32_t* __restrict__ lens, int B, int S, int vocab,
                                                       int max_row_bytes, long long text_bytes) {
  // + 16: the row starts up to 15 bytes into its first 16-B piece; + 32: a piece hash reads
  // 7 dwords from its aligned start (at most 28 bytes past a byte of the row)
  __shared__ __attribute__((aligned(16))) uint8_t rowbuf[4][kMaxRowBytes + 48];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int row = blockIdx.x * 4 + w;
  if (row >= B) return;
  const int start = offsets[row];
  const int n = min(offsets[row + 1] - start, max_row_bytes);
  // the row's bytes arrive as aligned 16-B pieces (one load per lane for a 1 KiB row;
  // byte loads were 16 dependent round trips), the row itself starts sh bytes in; the
  // last piece is clipped at the end of the text buffer
  const int a0 = start & ~15, sh = start - a0;
  for (int c = lane; c < (sh + n + 15) >> 4; c += 64) {
    const long long g = (long long)a0 + 16 * c;
    if (g + 16 <= text_bytes) {
      *reinterpret_cast<uint4*>(rowbuf[w] + 16 * c) = *reinterpret_cast<const uint4*>(text + g);
    } else {
      for (int k = 0; k < 16 && g + k < text_bytes; ++k) rowbuf[w][16 * c + k] = text[g + k];
    }
  }
  uint8_t* buf = rowbuf[w] + sh;
  // each wave reads only its own LDS slice: a wave-level fence suffices
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");

  const int cap = S - 2;
  const uint32_t mod = (uint32_t)(vocab - 1000);
  uint32_t cont_basis = fnv_step(fnv_step(kFnvBasis, '#'), '#');
  int32_t* out = ids + (size_t)row * S;
  int ntok = 0;
  int carry = 0;
  const uint8_t* rb = rowbuf[w];
  for (int base = 0; base < n && ntok < cap; base += 64) {
    const int i = base + lane;
    const int cls = i < n ? byte_class(buf[i]) : 0;
    const int cls2 = i + 64 < n ? byte_class(buf[i + 64]) : 0;
    const uint64_t W = __ballot(cls == 2), W2 = __ballot(cls2 == 2);
    int prev = __shfl_up(cls, 1, 64);
    if (lane == 0) prev = carry;
    const bool st = cls == 1 || (cls == 2 && prev != 2);
    int wlen = 0, npieces = 0;
    if (st) {
      if (cls == 1) {
        npieces = 1;
        wlen = 1;
      } else {
        // word bytes from i on: bits lane..63 of W, then W2
        const uint64_t x = lane == 0 ? W : ((W >> lane) | (W2 << (64 - lane)));
        if (~x != 0) {
          wlen = __builtin_ctzll(~x);
        } else {  // 64+ word bytes: walk the rest
          int j = i + 64;
          while (j < n && byte_class(buf[j]) == 2) ++j;
          wlen = j - i;
        }
        npieces = (wlen + kPiece - 1) / kPiece;
      }
    }
    const int incl = wave_inclusive_scan(npieces, lane);
    const int excl = incl - npieces;
    for (int p = 0;; ++p) {
      const bool act = st && p < npieces && ntok + excl + p < cap;
      if (__ballot(act) == 0) break;
      const int b0 = p * kPiece, len = min(wlen - b0, kPiece);  // this lane's piece: bytes [i+b0, +len)
      int lmax = act ? len : 0;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) lmax = max(lmax, __shfl_xor(lmax, o, 64));
      // 7 aligned dwords cover the piece (<= 24 bytes at offset <= 3); v_alignbyte drops the offset
      const int abs0 = sh + i + b0;
      const uint32_t* dp = reinterpret_cast<const uint32_t*>(rb + (act ? (abs0 & ~3) : 0));
      const uint32_t sft = (uint32_t)(abs0 & 3) * 8u;
      uint32_t d[7], e[6];
#pragma unroll
      for (int k = 0; k < 7; ++k) d[k] = dp[k];
#pragma unroll
      for (int k = 0; k < 6; ++k) e[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sft >> 3);
      uint32_t h = (cls == 1 || p == 0) ? kFnvBasis : cont_basis;
#pragma unroll
      for (int k = 0; k < kPiece; ++k) {
        if (k >= lmax) break;
        const uint32_t cb = (e[k >> 2] >> ((k & 3) * 8)) & 0xffu;
        const uint32_t hn = fnv_step(h, cb);
        h = k < len ? hn : h;
      }
      if (act) out[1 + ntok + excl + p] = (int32_t)(1000u + h % mod);
    }
    ntok += __shfl(incl, 63, 64);
    carry = __shfl(cls, 63, 64);
  }
  ntok = min(ntok, cap);
  if (lane == 0) {
    out[0] = 101;
    out[1 + ntok] = 102;
    lens[row] = ntok + 2;
  }
  for (int j = ntok + 2 + lane; j < S; j += 64) out[j] = 0;
}

}  // namespace

void tokenize_hash(const uint8_t* text, const int32_t* offsets, int32_t* ids, int32_t* lens, int B, int S, int vocab,
                   int max_row_bytes, hipStream_t stream, long long text_bytes) {
  ATPU_CHECK((reinterpret_cast<uintptr_t>(text) & 15) == 0, "tokenize: text buffer must be 16-byte aligned");
  ATPU_CHECK(S >= 2, "tokenize: S must be >= 2");
  ATPU_CHECK(vocab > 1000, "tokenize: vocab must exceed the 1000 reserved ids");
  ATPU_CHECK(max_row_bytes > 0 && max_row_bytes <= kMaxRowBytes, "tokenize: max_row_bytes must be in (0, 4096]");
  if (B <= 0) return;
  hipLaunchKernelGGL(tokenize_kernel, dim3((B + 3) / 4), dim3(256), 0, stream, text, offsets, ids, lens, B, S, vocab,
                     max_row_bytes, text_bytes);
  ATPU_HIP_CHECK(hipGetLastError());
}

}  // namespace atpu
