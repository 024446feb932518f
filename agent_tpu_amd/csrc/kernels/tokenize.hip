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
// per step: each lane classifies its byte, token starts are found against the
// left neighbour (shfl_up; chunk-carry through lane 63), the lane at a word
// start walks its word in LDS to count/hash pieces, and an inclusive wave scan
// of piece counts gives every token its output slot. The scan stops as soon
// as S-2 tokens exist, so long rows cost only the bytes that are used.
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
  __shared__ __attribute__((aligned(16))) uint8_t rowbuf[4][kMaxRowBytes + 16];
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
  for (int base = 0; base < n && ntok < cap; base += 64) {
    const int i = base + lane;
    const int cls = i < n ? byte_class(buf[i]) : 0;
    int prev = __shfl_up(cls, 1, 64);
    if (lane == 0) prev = carry;
    const bool st = cls == 1 || (cls == 2 && prev != 2);
    int wlen = 0, npieces = 0;
    if (st) {
      if (cls == 1) {
        npieces = 1;
      } else {
        int j = i;
        while (j < n && byte_class(buf[j]) == 2) ++j;
        wlen = j - i;
        npieces = (wlen + kPiece - 1) / kPiece;
      }
    }
    const int incl = wave_inclusive_scan(npieces, lane);
    const int excl = incl - npieces;
    if (st) {
      for (int p = 0; p < npieces; ++p) {
        const int pos = ntok + excl + p;
        if (pos >= cap) break;
        uint32_t h;
        if (cls == 1) {
          h = fnv_step(kFnvBasis, buf[i]);
        } else {
          h = p == 0 ? kFnvBasis : cont_basis;
          const int b0 = i + p * kPiece, b1 = min(i + (p + 1) * kPiece, i + wlen);
          for (int j = b0; j < b1; ++j) h = fnv_step(h, buf[j]);
        }
        out[1 + pos] = (int32_t)(1000u + h % mod);
      }
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
