// MFMA GEMM for every dense projection of the MaPLe towers (SURVEY.md §2.2 K1, K5, K7-K10 and
// their dX / dW backward products).
//
//   C[M,N] = epilogue( A[M,K] . B[N,K]^T )      A, B fp16 row-major (K contiguous), fp32 accumulate
//
// This "NT" form is the nn.Linear forward layout (weight [out,in]); dX products use a
// pre-transposed weight copy and dW products use transposed activations, so one kernel family
// serves all of them.  Epilogues reproduce the reference's fp16 rounding points
// (torch addmm on fp16 rounds acc+bias once; the residual add and QuickGELU round per op).
//
// Structure (gfx950): 256 threads = 4 waves (2x2), each wave a (BM/2)x(BN/2) tile of
// v_mfma_f32_16x16x32_f16; BK = 64; LDS double buffer with a 16-B-chunk XOR swizzle
// (chunk ^ (row & 7)) so ds_read_b128 fragment reads are conflict-free; register-staged
// global loads for tile k+1 issued before the MFMAs of tile k and written to LDS after them;
// one barrier per K-step; XCD-aware bijective block remap so tiles sharing an A panel share
// an L2.  The MFMA is issued "swapped" (weight fragment as the A operand) so each lane ends with
// 4 consecutive output columns of one row -> 8-byte stores.
#include "mf_common.h"

namespace {

enum Epi : int {
  EPI_NONE = 0,        // C = fp16(acc)
  EPI_BIAS = 1,        // C = fp16(acc + bias)
  EPI_BIAS_RESID = 2,  // C = fp16(R + fp16(acc + bias))        (R = aux_in, may alias C)
  EPI_BIAS_GELU = 3,   // F = fp16(acc + bias) -> aux_out ; C = QuickGELU16(F)
  EPI_DGELU = 4,       // dG = fp16(acc) ; C = QuickGELU16_bwd(dG, F = aux_in)
  EPI_F32 = 5,         // C(float) = acc
  EPI_RESID = 6,       // C = fp16(R + fp16(acc))               (no bias)
};

struct GemmArgs {
  const f16* A;
  const f16* B;
  void* C;
  const f16* bias;
  const f16* aux_in;
  f16* aux_out;
  int64_t lda, ldb, ldc, ld_aux;
  int M, N, K;
};

constexpr int BK = 64;

MF_DEV int swz(int row, int chunk) { return chunk ^ (row & 7); }

template <int BM, int BN, int EPI>
__global__ __launch_bounds__(256, 2) void gemm_nt_kernel(GemmArgs g) {
  constexpr int WM = BM / 2, WN = BN / 2;
  constexpr int TM = WM / 16, TN = WN / 16;
  constexpr int A_CH = BM * 8 / 256;  // 16-B chunks per thread per A tile
  constexpr int B_CH = BN * 8 / 256;
  __shared__ __attribute__((aligned(16))) f16 lds[2 * (BM + BN) * BK];
  f16* ldsA = lds;
  f16* ldsB = lds + 2 * BM * BK;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wid >> 1, wave_n = wid & 1;

  // XCD-aware bijective remap (cdna_hip_programming.md §5 'XCD swizzle must be bijective')
  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int m0 = (wgid / tiles_n) * BM;
  const int n0 = (wgid % tiles_n) * BN;

  // staging coordinates
  const int st_c = tid & 7;
  const int st_r = tid >> 3;  // 0..31
  const f16* a_src[A_CH];
  const f16* b_src[B_CH];
#pragma unroll
  for (int i = 0; i < A_CH; ++i) {
    int row = m0 + st_r + 32 * i;
    row = row < g.M ? row : g.M - 1;
    a_src[i] = g.A + (int64_t)row * g.lda + st_c * 8;
  }
#pragma unroll
  for (int i = 0; i < B_CH; ++i) {
    int row = n0 + st_r + 32 * i;
    row = row < g.N ? row : g.N - 1;
    b_src[i] = g.B + (int64_t)row * g.ldb + st_c * 8;
  }
  f16x8 ra[A_CH], rb[B_CH];

  auto load_regs = [&](int k0) {
#pragma unroll
    for (int i = 0; i < A_CH; ++i) ra[i] = *(const f16x8*)(a_src[i] + k0);
#pragma unroll
    for (int i = 0; i < B_CH; ++i) rb[i] = *(const f16x8*)(b_src[i] + k0);
  };
  auto write_lds = [&](int buf) {
    f16* la = ldsA + buf * BM * BK;
    f16* lb = ldsB + buf * BN * BK;
#pragma unroll
    for (int i = 0; i < A_CH; ++i) {
      int row = st_r + 32 * i;
      *(f16x8*)(la + row * BK + swz(row, st_c) * 8) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < B_CH; ++i) {
      int row = st_r + 32 * i;
      *(f16x8*)(lb + row * BK + swz(row, st_c) * 8) = rb[i];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  load_regs(0);
  write_lds(0);
  __syncthreads();

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_regs((kt + 1) * BK);
    const f16* la = ldsA + cur * BM * BK;
    const f16* lb = ldsB + cur * BN * BK;
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      f16x8 af[TM], bf[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        int row = wave_m * WM + i * 16 + fr;
        af[i] = *(const f16x8*)(la + row * BK + swz(row, 4 * s + fg) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        int row = wave_n * WN + j * 16 + fr;
        bf[j] = *(const f16x8*)(lb + row * BK + swz(row, 4 * s + fg) * 8);
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) write_lds(cur ^ 1);
    __syncthreads();
  }

  // epilogue: lane holds C[m = .. + fr][n = .. + 4*fg + e], e = 0..3
#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int m = m0 + wave_m * WM + i * 16 + fr;
    if (m >= g.M) continue;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int n = n0 + wave_n * WN + j * 16 + 4 * fg;
      if (n >= g.N) continue;
      f32x4 v = acc[i][j];
      if constexpr (EPI == EPI_F32) {
        *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = v;
      } else {
        f16x4 out;
        if constexpr (EPI == EPI_NONE) {
#pragma unroll
          for (int e = 0; e < 4; ++e) out[e] = (f16)v[e];
        } else if constexpr (EPI == EPI_BIAS) {
          f16x4 b = *(const f16x4*)(g.bias + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) out[e] = (f16)(v[e] + (float)b[e]);
        } else if constexpr (EPI == EPI_BIAS_RESID) {
          f16x4 b = *(const f16x4*)(g.bias + n);
          f16x4 rr = *(const f16x4*)(g.aux_in + (int64_t)m * g.ld_aux + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) out[e] = (f16)((float)rr[e] + r16(v[e] + (float)b[e]));
        } else if constexpr (EPI == EPI_RESID) {
          f16x4 rr = *(const f16x4*)(g.aux_in + (int64_t)m * g.ld_aux + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) out[e] = (f16)((float)rr[e] + r16(v[e]));
        } else if constexpr (EPI == EPI_BIAS_GELU) {
          f16x4 b = *(const f16x4*)(g.bias + n);
          f16x4 fo;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            float f = r16(v[e] + (float)b[e]);
            float t2;
            fo[e] = (f16)f;
            out[e] = (f16)quick_gelu16(f, &t2);
          }
          *(f16x4*)(g.aux_out + (int64_t)m * g.ld_aux + n) = fo;
        } else if constexpr (EPI == EPI_DGELU) {
          f16x4 ff = *(const f16x4*)(g.aux_in + (int64_t)m * g.ld_aux + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) out[e] = (f16)quick_gelu16_bwd(r16(v[e]), (float)ff[e]);
        }
        *(f16x4*)((f16*)g.C + (int64_t)m * g.ldc + n) = out;
      }
    }
  }
}

template <int BM, int BN>
int launch_tile(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles), block(256);
  switch (epi) {
    case EPI_NONE: gemm_nt_kernel<BM, BN, EPI_NONE><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: gemm_nt_kernel<BM, BN, EPI_BIAS><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RESID: gemm_nt_kernel<BM, BN, EPI_BIAS_RESID><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm_nt_kernel<BM, BN, EPI_BIAS_GELU><<<grid, block, 0, st>>>(a); break;
    case EPI_DGELU: gemm_nt_kernel<BM, BN, EPI_DGELU><<<grid, block, 0, st>>>(a); break;
    case EPI_F32: gemm_nt_kernel<BM, BN, EPI_F32><<<grid, block, 0, st>>>(a); break;
    case EPI_RESID: gemm_nt_kernel<BM, BN, EPI_RESID><<<grid, block, 0, st>>>(a); break;
    default: return mf_set_error("mf_gemm_nt: bad epilogue", -2);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

}  // namespace

extern "C" int mf_gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                          int N, int K, const void* bias, const void* aux_in, void* aux_out, int64_t ld_aux,
                          int epilogue, int tile, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  if (K <= 0 || (K % BK) != 0) return mf_set_error("mf_gemm_nt: K must be a positive multiple of 64", -1);
  if ((N % 4) != 0 || (lda % 8) || (ldb % 8) || (ldc % 4)) return mf_set_error("mf_gemm_nt: alignment", -1);
  if ((epilogue == EPI_BIAS || epilogue == EPI_BIAS_RESID || epilogue == EPI_BIAS_GELU) && !bias)
    return mf_set_error("mf_gemm_nt: epilogue needs bias", -1);
  if ((epilogue == EPI_BIAS_RESID || epilogue == EPI_DGELU || epilogue == EPI_RESID) && !aux_in)
    return mf_set_error("mf_gemm_nt: epilogue needs aux_in", -1);
  if (epilogue == EPI_BIAS_GELU && !aux_out) return mf_set_error("mf_gemm_nt: epilogue needs aux_out", -1);
  GemmArgs a{(const f16*)A, (const f16*)B, C, (const f16*)bias, (const f16*)aux_in, (f16*)aux_out,
             lda, ldb, ldc, ld_aux, M, N, K};
  hipStream_t st = (hipStream_t)stream;
  if (tile == 0) {  // heuristic: fill the 256 CUs
    int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
    tile = t128 >= 512 ? 1 : (t128 >= 128 ? 2 : 3);
  }
  switch (tile) {
    case 1: return launch_tile<128, 128>(a, epilogue, st);
    case 2: return launch_tile<128, 64>(a, epilogue, st);
    case 3: return launch_tile<64, 64>(a, epilogue, st);
    default: return mf_set_error("mf_gemm_nt: bad tile id", -2);
  }
}
