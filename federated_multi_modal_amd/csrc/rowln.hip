// Fused out-projection + residual + LayerNorm of a residual block (clip/model.py:303-305, 350-351 and
// 153-159): X1 = fp16(X + fp16(O . W_out^T + b_out)) and h2 = ln_2(X1), with its row mean / rstd, in one
// launch instead of mf_gemm_nt(EPI_BIAS_RESID) + mf_layernorm_fwd.
//
// Full-row tiles: a workgroup owns BM rows x all N (= 768) columns, so the LayerNorm's row statistics need
// no second pass over HBM and no second launch.  The K loop streams W_out [N][K] through LDS (a 3-stage
// ring of 32-deep K-steps by LDS-DMA: BM x 32 of A and N x 32 of W per stage); each of the 8 waves owns
// N/8 columns.  The epilogue stages X1 in LDS and then runs ln_fwd2_kernel's per-row arithmetic (the same
// lane layout and reduction order) on it, so X1, h2, mean and rstd are bit-identical to the two-launch pair:
// the MFMAs accumulate every output over k in the same ascending 32-k order as every mf_gemm tile, and the
// epilogue rounds at the same points (fp16(acc + b), then fp16(X + that)).
#include <cstdlib>

#include "mf_common.h"

namespace {

typedef __attribute__((address_space(3))) void* lds_ptr_t;

constexpr int RL_BK = 32;     // K per stage: one v_mfma_f32_16x16x32_f16 k-sub
constexpr int RL_STAGES = 3;  // ring depth (two stages in flight)

// 16-byte chunk position of chunk c of image row r (rows of 32 fp16 = 4 chunks): rows r, r+4, r+8, r+12
// take the four positions, so the 16 rows of a ds_read_b128 lane group cover all 64 banks once
MF_DEV int rl_pos(int r, int c) { return c ^ ((r >> 2) & 3); }

MF_DEV float rl_half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int BM, int N>
__global__ __launch_bounds__(512) void gemm_rowln_kernel(const f16* __restrict__ A, int64_t lda,
                                                         const f16* __restrict__ W, int64_t ldw,
                                                         const f16* __restrict__ bias, const f16* __restrict__ R,
                                                         int64_t ldr, f16* __restrict__ C, int64_t ldc,
                                                         const float* __restrict__ gamma,
                                                         const float* __restrict__ beta, f16* __restrict__ Y,
                                                         int64_t ldy, float* __restrict__ mean_out,
                                                         float* __restrict__ rstd_out, int M, int K) {
  constexpr int NW = 8;
  constexpr int WN = N / NW;  // columns per wave
  constexpr int CB = WN / 16;
  constexpr int RB = BM / 16;
  constexpr int A_ELEMS = BM * RL_BK, B_ELEMS = N * RL_BK, STAGE = A_ELEMS + B_ELEMS;
  constexpr int A_INS = BM / 16, B_INS = N / 16;  // 1 KB LDS-DMA wave instructions (16 rows x 64 B) per stage
  constexpr int B_PER_W = B_INS / NW;
  constexpr int LDX = N + 8;  // X1 staging pitch (fp16)
  constexpr int LDS_ELEMS = RL_STAGES * STAGE > BM * LDX ? RL_STAGES * STAGE : BM * LDX;
  constexpr int CH = N / 256;  // 16-byte chunks per half-wave lane in the LayerNorm phase
  static_assert(WN % 16 == 0 && B_INS % NW == 0 && A_INS <= NW && N % 256 == 0, "shape");
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(16))) f16 lds[LDS_ELEMS];

  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m0 = blockIdx.x * BM;
  const int fr = lane & 15, fg = lane >> 4;

  const __amdgpu_buffer_rsrc_t a_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, (int)(((int64_t)(M - 1) * lda + K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc =
      __builtin_amdgcn_make_buffer_rsrc((void*)W, 0, (int)(((int64_t)(N - 1) * ldw + K) * 2), 0x00020000);
  // this lane's 16 bytes of an instruction covering image rows r0 .. r0+15: row r0 + lane/4, LDS position
  // lane%4, which holds chunk rl_pos(row, lane%4) (the swizzle is its own inverse)
  const int lrow = lane >> 2, lpos = lane & 3;
  auto issue = [&](int kt) {
    f16* st = lds + (kt % RL_STAGES) * STAGE;
    const int k0 = kt * RL_BK;
    if (w < A_INS) {
      const int r = w * 16 + lrow;
      const int voff = (int)(((int64_t)(m0 + r) * lda + k0 + 8 * rl_pos(r, lpos)) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr_t)(st + w * 16 * RL_BK), 16, voff, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < B_PER_W; ++i) {
      const int r0 = (w * B_PER_W + i) * 16, r = r0 + lrow;
      const int voff = (int)(((int64_t)r * ldw + k0 + 8 * rl_pos(r, lpos)) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr_t)(st + A_ELEMS + r0 * RL_BK), 16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[RB][CB];
#pragma unroll
  for (int i = 0; i < RB; ++i)
#pragma unroll
    for (int j = 0; j < CB; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int nk = K / RL_BK;
  const int wcol = w * WN;
  issue(0);
  if (nk > 1) issue(1);
#pragma unroll 1
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (this wave's share; stage kt+1, when issued, may still be in flight)
    if (kt + 1 < nk) {
      if (w < A_INS) __builtin_amdgcn_s_waitcnt((B_PER_W + 1) | (7 << 4) | (15 << 8));
      else __builtin_amdgcn_s_waitcnt(B_PER_W | (7 << 4) | (15 << 8));
    } else {
      __builtin_amdgcn_s_waitcnt(0 | (7 << 4) | (15 << 8));
    }
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_barrier();  // every wave's stage-kt bytes landed; every wave done with stage kt-1
    asm volatile("" ::: "memory");
    if (kt + 2 < nk) issue(kt + 2);  // into stage kt-1's buffer
    const f16* st = lds + (kt % RL_STAGES) * STAGE;
    f16x8 af[RB], bf[CB];
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int r = i * 16 + fr;
      af[i] = *(const f16x8*)(st + r * RL_BK + 8 * rl_pos(r, fg));
    }
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const int r = wcol + j * 16 + fr;
      bf[j] = *(const f16x8*)(st + A_ELEMS + r * RL_BK + 8 * rl_pos(r, fg));
    }
#pragma unroll
    for (int i = 0; i < RB; ++i)
#pragma unroll
      for (int j = 0; j < CB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
  }
  __syncthreads();  // every wave done with the ring (no LDS-DMA in flight after the last wait)

  // epilogue 1: X1 = fp16(R + fp16(acc + b)) into the LDS staging tile; acc[i][j][e] holds
  // C[m0 + 16 i + fr][wcol + 16 j + 4 fg + e]
  f16* X = lds;
#pragma unroll
  for (int j = 0; j < CB; ++j) {
    const int n = wcol + j * 16 + 4 * fg;
    const f16x4 bv = *(const f16x4*)(bias + n);
#pragma unroll
    for (int i = 0; i < RB; ++i) {
      const int ml = i * 16 + fr;
      const int64_t m = m0 + ml;
      f16x4 out = {};
      if (m < M) {
        const f16x4 rv = *(const f16x4*)(R + m * ldr + n);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const f16 t = (f16)(acc[i][j][e] + (float)bv[e]);
          out[e] = (f16)((float)rv[e] + (float)t);
        }
      }
      *(f16x4*)(X + ml * LDX + n) = out;
    }
  }
  __syncthreads();

  // epilogue 2: per row, X1 out and ln_fwd2_kernel's arithmetic (half-wave per row, 16-byte chunks,
  // statistics by 32-lane butterflies in its order)
  const int hw = tid >> 5, hl = tid & 31;
  for (int row = hw; row < BM; row += 2 * NW) {
    const int64_t m = m0 + row;
    if (m >= M) break;  // whole half-waves leave together
    f16x8 t[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      t[j] = *(const f16x8*)(X + row * LDX + 8 * (hl + 32 * j));
      *(f16x8*)(C + m * ldc + 8 * (hl + 32 * j)) = t[j];
    }
    float v[CH * 8];
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[j * 8 + e] = (float)t[j][e];
        if (e < 4) s0 += v[j * 8 + e];
        else s1 += v[j * 8 + e];
      }
    const float mean = (rl_half_sum(s0) + rl_half_sum(s1)) / (float)N;
    float ss0 = 0.f, ss1 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[j * 8 + e] - mean;
        if (e < 4) ss0 += d * d;
        else ss1 += d * d;
      }
    const float var = (rl_half_sum(ss0) + rl_half_sum(ss1)) / (float)N;
    const float rstd = 1.0f / sqrtf(fmaxf(var, 0.f) + 1e-5f);
    const float bias2 = -rstd * mean;
    f16* yr = Y + m * ldy;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = 8 * (hl + 32 * j);
      const f32x4 g0 = *(const f32x4*)(gamma + c), g1 = *(const f32x4*)(gamma + c + 4);
      const f32x4 b0 = *(const f32x4*)(beta + c), b1 = *(const f32x4*)(beta + c + 4);
      f16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float tt = v[j * 8 + e] * rstd;
        tt = tt + bias2;
        tt = tt * (e < 4 ? g0[e] : g1[e - 4]);
        tt = tt + (e < 4 ? b0[e] : b1[e - 4]);
        o[e] = (f16)tt;
      }
      *(f16x8*)(yr + c) = o;
    }
    if (hl == 0) {
      if (mean_out) mean_out[m] = mean;
      if (rstd_out) rstd_out[m] = rstd;
    }
  }
}

inline int rowln_bm() {  // rows per workgroup (MAPFED_ROWLN_BM=32 / 64, A/B knob)
  static const int b = getenv("MAPFED_ROWLN_BM") ? atoi(getenv("MAPFED_ROWLN_BM")) : 64;
  return b == 32 ? 32 : 64;
}

}  // namespace

extern "C" int mf_gemm_resid_ln_supported(int N, int K) { return N == 768 && K > 0 && K % RL_BK == 0; }

// X1[M,N] = fp16(R + fp16(A[M,K] . W[N,K]^T + bias)), Y = LayerNorm(X1) (fp32 gamma / beta, eps 1e-5), row mean /
// rstd: mf_gemm_nt(EPI_BIAS_RESID) + mf_layernorm_fwd in one launch, bit-identical.  N = 768, K % 32 == 0.
extern "C" int mf_gemm_resid_ln(const void* A, int64_t lda, const void* W, int64_t ldw, const void* bias,
                                const void* R, int64_t ldr, void* C, int64_t ldc, const float* gamma, const float* beta,
                                void* Y, int64_t ldy, float* mean, float* rstd, int M, int N, int K, void* stream) {
  if (M <= 0) return 0;
  if (!mf_gemm_resid_ln_supported(N, K)) return mf_set_error("mf_gemm_resid_ln: N = 768 and K % 32 == 0", -1);
  if ((lda % 8) || (ldw % 8) || (ldr % 8) || (ldc % 8) || (ldy % 8) || lda < K || ldw < K || ldr < N || ldc < N ||
      ldy < N || (uintptr_t)A % 16 || (uintptr_t)W % 16 || (uintptr_t)R % 16 || (uintptr_t)C % 16 ||
      (uintptr_t)Y % 16 || (uintptr_t)bias % 8 || (uintptr_t)gamma % 16 || (uintptr_t)beta % 16)
    return mf_set_error("mf_gemm_resid_ln: strides / alignment", -1);
  if (((int64_t)(M - 1) * lda + K) * 2 > INT32_MAX || ((int64_t)(N - 1) * ldw + K) * 2 > INT32_MAX)
    return mf_set_error("mf_gemm_resid_ln: operand exceeds the 2 GB buffer range", -1);
  hipStream_t st = (hipStream_t)stream;
  if (rowln_bm() == 32)
    gemm_rowln_kernel<32, 768><<<(M + 31) / 32, 512, 0, st>>>(
        (const f16*)A, lda, (const f16*)W, ldw, (const f16*)bias, (const f16*)R, ldr, (f16*)C, ldc, gamma, beta,
        (f16*)Y, ldy, mean, rstd, M, K);
  else
    gemm_rowln_kernel<64, 768><<<(M + 63) / 64, 512, 0, st>>>(
        (const f16*)A, lda, (const f16*)W, ldw, (const f16*)bias, (const f16*)R, ldr, (f16*)C, ldc, gamma, beta,
        (f16*)Y, ldy, mean, rstd, M, K);
  MF_CHECK_LAUNCH();
  return 0;
}
