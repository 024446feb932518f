// Fused masked multi-head attention (T5 encoder/cross
// attention reuses it with an additive position bias and scale 1).
//
//   O[b,q,h,:] = softmax_k( scale * Q[b,q,h]·K[b,k,h] + bias[h,q,k] ) · V[b,k,h,:]
//   keys k >= lens[b] are masked; causal=1 additionally masks k > q.
//
// D = 64 (BERT-base/large, T5-base). Workgroup = 4 waves = 128 queries of one
// (batch, head); each wave owns 32 queries. Keys are processed in chunks of
// 128 with an fp32 online softmax, so any Skv works; BERT (S=128) is one chunk.
//
// CDNA4 mapping (cdna_hip_programming.md §3, App. B "Fused attention"):
//  * S^T = K·Q^T on v_mfma_f32_16x16x32_bf16: the KEY index sits in the
//    accumulator rows and the QUERY on the lane, so every lane owns whole
//    score columns -> row max / row sum are in-register plus two xor-shuffles,
//    and the P^T tile is ALREADY the B operand of O^T = V^T·P^T (the k order
//    inside a 32-key step is permuted identically on both operands).
//  * K chunk staged by global_load_lds (16 B/lane) into a row-swizzled image
//    (chunk ^ ((row>>1)&7)) read conflict-free with ds_read_b128.
//  * V chunk staged transposed, V^T[d][key], with 8-byte slots swizzled by
//    (key>>2) ^ ((d&15)<<1): the PV A-operand reads (ds_read_b64, 16 d-rows x
//    2 key groups per half-wave) hit 32 distinct slots -> conflict-free.
//  * Q fragments go global -> VGPR directly (read once per wave).
#include "atpu/common.h"
#include "atpu/kernels.h"

namespace atpu {
namespace {

constexpr int kD = 64;
constexpr int kKC = 128;  // keys per chunk
constexpr int kQB = 128;  // queries per workgroup
constexpr int kKRowB = kD * 2;     // 128 B per K row
constexpr int kVtRowB = kKC * 2;   // 256 B per V^T row
constexpr int kLdsK = kKC * kKRowB;  // 16 KiB
constexpr int kLdsV = kD * kVtRowB;  // 16 KiB

__device__ __forceinline__ int kswz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }
// byte offset of V^T[d][key] (key in [0,128))
__device__ __forceinline__ int vt_off(int d, int key) {
  return d * kVtRowB + ((((key >> 2) ^ ((d & 15) << 1))) << 3) + ((key & 3) << 1);
}

__global__ __launch_bounds__(256, 2) void attention_fwd_kernel(
    const bf16* __restrict__ Q, int ldq, const bf16* __restrict__ Kp, int ldk, const bf16* __restrict__ V, int ldv,
    bf16* __restrict__ O, int ldo, const int32_t* __restrict__ lens, const float* __restrict__ bias, int Sq, int Skv,
    int H, float scale, int causal) {
  __shared__ __attribute__((aligned(16))) char lds[kLdsK + kLdsV];
  char* ldsK = lds;
  char* ldsV = lds + kLdsK;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int len = lens ? min(lens[b], Skv) : Skv;
  const int fr = lane & 15, fg = lane >> 4;

  const bf16* Qb = Q + (size_t)b * Sq * ldq + h * kD;
  const bf16* Kb = Kp + (size_t)b * Skv * ldk + h * kD;
  const bf16* Vb = V + (size_t)b * Skv * ldv + h * kD;

  // ---- this wave's Q fragments: 2 query tiles x 2 d-steps, 16 B each ----
  const int qw = qblk * kQB + wave * 32;
  bf16x8 qf[2][2];
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = min(qw + qt * 16 + fr, Sq - 1);
#pragma unroll
    for (int ds = 0; ds < 2; ++ds) qf[qt][ds] = *reinterpret_cast<const bf16x8*>(Qb + (size_t)q * ldq + ds * 32 + fg * 8);
  }

  float m_run[2], l_run[2];
  f32x4 o[4][2];  // O^T tiles [d-tile][q-tile]
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    m_run[qt] = -1e30f;
    l_run[qt] = 0.f;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt][qt] = f32x4{0.f, 0.f, 0.f, 0.f};
  }

  const int kv_end = causal ? min(len, qblk * kQB + kQB) : len;
  for (int kc = 0; kc < kv_end; kc += kKC) {
    __syncthreads();  // previous chunk fully consumed
    // ---- stage K chunk: 16 wave-instructions of 8 rows (4 per wave) ----
    {
      const int srow = lane >> 3, spos = lane & 7;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = (i * 4 + wave) * 8 + srow;
        const int key = min(kc + r, Skv - 1);
        glds16(Kb + (size_t)key * ldk + kswz(r, spos) * 8, ldsK + (i * 4 + wave) * 8 * kKRowB);
      }
    }
    // ---- stage V chunk transposed: thread -> (key, 8 d) pieces ----
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int piece = i * 256 + tid;  // 1024 pieces = 128 keys x 8 d-groups
      const int key = piece >> 3, dg = (piece & 7) * 8;
      const int gk = min(kc + key, Skv - 1);
      const bf16x8 v = *reinterpret_cast<const bf16x8*>(Vb + (size_t)gk * ldv + dg);
#pragma unroll
      for (int e = 0; e < 8; ++e) *reinterpret_cast<bf16*>(ldsV + vt_off(dg + e, key)) = v[e];
    }
    wait_vmcnt0();
    __syncthreads();

    // ---- S^T = K·Q^T : s[kt][qt] holds keys kt*16 + fg*4 + r, query fr ----
    f32x4 s[8][2];
#pragma unroll
    for (int kt = 0; kt < 8; ++kt) {
      s[kt][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      s[kt][1] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ds = 0; ds < 2; ++ds) {
        const int r = kt * 16 + fr;
        const bf16x8 kf = *reinterpret_cast<const bf16x8*>(ldsK + r * kKRowB + kswz(r, ds * 4 + fg) * 16);
        s[kt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[0][ds], s[kt][0], 0, 0, 0);
        s[kt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(kf, qf[1][ds], s[kt][1], 0, 0, 0);
      }
    }

    // ---- scale, bias, mask, online softmax (per query column) ----
#pragma unroll
    for (int qt = 0; qt < 2; ++qt) {
      const int q = qw + qt * 16 + fr;
      const int qc = min(q, Sq - 1);
      float cmax = -1e30f;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt) {
        const int key0 = kc + kt * 16 + fg * 4;
        f32x4 bv = f32x4{0.f, 0.f, 0.f, 0.f};
        if (bias && key0 < Skv) {
          // Skv % 4 == 0 is enforced on the host for the bias path
          bv = *reinterpret_cast<const f32x4*>(bias + ((size_t)h * Sq + qc) * Skv + key0);
        }
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int key = key0 + r;
          float x = s[kt][qt][r] * scale + bv[r];
          const bool dead = key >= len || (causal && key > q);
          x = dead ? -1e30f : x;
          s[kt][qt][r] = x;
          cmax = fmaxf(cmax, x);
        }
      }
      cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
      cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
      const float m_new = fmaxf(m_run[qt], cmax);
      const float alpha = __expf(m_run[qt] - m_new);
      float psum = 0.f;
#pragma unroll
      for (int kt = 0; kt < 8; ++kt)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float x = s[kt][qt][r];
          const float p = x <= -1e29f ? 0.f : __expf(x - m_new);
          s[kt][qt][r] = p;
          psum += p;
        }
      psum += __shfl_xor(psum, 16, 64);
      psum += __shfl_xor(psum, 32, 64);
      l_run[qt] = l_run[qt] * alpha + psum;
      m_run[qt] = m_new;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) o[dt][qt] *= alpha;
    }

    // ---- O^T += V^T · P^T over 4 key-steps of 32 ----
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 pf[2];
#pragma unroll
      for (int qt = 0; qt < 2; ++qt)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          pf[qt][e] = f2bf(s[2 * ks][qt][e]);
          pf[qt][4 + e] = f2bf(s[2 * ks + 1][qt][e]);
        }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        const int d = dt * 16 + fr;
        const bf16x4 lo = *reinterpret_cast<const bf16x4*>(ldsV + vt_off(d, ks * 32 + fg * 4));
        const bf16x4 hi = *reinterpret_cast<const bf16x4*>(ldsV + vt_off(d, ks * 32 + 16 + fg * 4));
        bf16x8 vf;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          vf[e] = lo[e];
          vf[4 + e] = hi[e];
        }
        o[dt][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[0], o[dt][0], 0, 0, 0);
        o[dt][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(vf, pf[1], o[dt][1], 0, 0, 0);
      }
    }
  }

  // ---- normalise and store: lane holds O[q][dt*16 + fg*4 + 0..3] ----
#pragma unroll
  for (int qt = 0; qt < 2; ++qt) {
    const int q = qw + qt * 16 + fr;
    if (q >= Sq) continue;
    const float inv = l_run[qt] > 0.f ? 1.f / l_run[qt] : 0.f;
    bf16* orow = O + ((size_t)b * Sq + q) * ldo + h * kD;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      bf16x4 v;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = f2bf(o[dt][qt][e] * inv);
      *reinterpret_cast<bf16x4*>(orow + dt * 16 + fg * 4) = v;
    }
  }
}

}  // namespace

void attention_fwd_strided(const bf16* q, int ldq, const bf16* k, int ldk, const bf16* v, int ldv, bf16* out,
                           int ldo, const int32_t* lens, const float* bias, int B, int Sq, int Skv, int H, int D,
                           float scale, int causal, hipStream_t stream) {
  ATPU_CHECK(D == kD, "attention: head dim must be 64");
  ATPU_CHECK(B > 0 && Sq > 0 && Skv > 0 && H > 0, "attention: empty problem");
  ATPU_CHECK(ldq % 8 == 0 && ldk % 8 == 0 && ldv % 8 == 0 && ldo % 4 == 0, "attention: row strides must be 16-B");
  ATPU_CHECK(!bias || Skv % 4 == 0, "attention: bias path needs Skv % 4 == 0");
  const dim3 grid((Sq + kQB - 1) / kQB, H, B);
  hipLaunchKernelGGL(attention_fwd_kernel, grid, dim3(256), 0, stream, q, ldq, k, ldk, v, ldv, out, ldo, lens, bias,
                     Sq, Skv, H, scale, causal);
  ATPU_HIP_CHECK(hipGetLastError());
}

void attention_fwd(const bf16* qkv, const int32_t* lens, const float* bias, bf16* out, int B, int S, int H, int D,
                   float scale, hipStream_t stream) {
  const int hd = H * D;
  attention_fwd_strided(qkv, 3 * hd, qkv + hd, 3 * hd, qkv + 2 * hd, 3 * hd, out, hd, lens, bias, B, S, S, H, D,
                        scale, 0, stream);
}

}  // namespace atpu
