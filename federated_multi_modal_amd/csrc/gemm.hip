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
  int vec8;  // C / aux row strides are multiples of 8 elements -> 16-byte epilogue accesses
};

// Elementwise epilogue on 8 consecutive columns (fp16 staged value t = the GEMM result rounded at
// the reference's first rounding point: fp16(acc + bias) or fp16(acc)).
template <int EPI>
MF_DEV void epi8(const GemmArgs& g, int64_t m, int n, int cnt, const f16* t) {
  f16* crow = (f16*)g.C + m * g.ldc + n;
  if (cnt == 8 && g.vec8) {
    f16x8 tv = *(const f16x8*)t;
    f16x8 out;
    if constexpr (EPI == EPI_NONE || EPI == EPI_BIAS) {
      out = tv;
    } else if constexpr (EPI == EPI_BIAS_RESID || EPI == EPI_RESID) {
      f16x8 rr = *(const f16x8*)(g.aux_in + m * g.ld_aux + n);
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = (f16)((float)rr[e] + (float)tv[e]);
    } else if constexpr (EPI == EPI_BIAS_GELU) {
      *(f16x8*)(g.aux_out + m * g.ld_aux + n) = tv;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t2;
        out[e] = (f16)quick_gelu16((float)tv[e], &t2);
      }
    } else if constexpr (EPI == EPI_DGELU) {
      f16x8 ff = *(const f16x8*)(g.aux_in + m * g.ld_aux + n);
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = (f16)quick_gelu16_bwd((float)tv[e], (float)ff[e]);
    }
    *(f16x8*)crow = out;
    return;
  }
  for (int e = 0; e < cnt; ++e) {
    const float tvv = (float)t[e];
    float o;
    if constexpr (EPI == EPI_NONE || EPI == EPI_BIAS) {
      o = tvv;
    } else if constexpr (EPI == EPI_BIAS_RESID || EPI == EPI_RESID) {
      o = (float)g.aux_in[m * g.ld_aux + n + e] + tvv;
    } else if constexpr (EPI == EPI_BIAS_GELU) {
      float t2;
      g.aux_out[m * g.ld_aux + n + e] = (f16)tvv;
      o = quick_gelu16(tvv, &t2);
    } else if constexpr (EPI == EPI_DGELU) {
      o = quick_gelu16_bwd(tvv, (float)g.aux_in[m * g.ld_aux + n + e]);
    }
    crow[e] = (f16)o;
  }
}

constexpr int BK = 64;

MF_DEV int swz(int row, int chunk) { return chunk ^ (row & 7); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4]<<14)
template <int N>
MF_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Tile BM x BN, (WM x WN) waves each owning a (BM/WM) x (BN/WN) block of 16x16 MFMA tiles, BK = 64.
// Operands go HBM -> LDS by global_load_lds (16 B per lane, no VGPR round trip): each wave
// instruction fills 8 rows x 128 B of the [rows][64] fp16 image; the 16-B-chunk XOR swizzle
// (chunk ^ (row & 7)) is applied to the per-lane SOURCE address (the LDS side is lane-linear), so
// the ds_read_b128 fragment reads stay conflict-free.  Two LDS buffers: the loads of K-step t+1
// are issued before the fragment reads + MFMAs of step t and drained by one vmcnt(0) + barrier
// per step (cdna_hip_programming.md §5.5 T3/T4 minimum 2-phase form).
template <int BM, int BN, int WM, int WN, int S, int EPI, bool PRIO = false>
__global__ __launch_bounds__(WM * WN * 64) void gemm_nt_kernel(GemmArgs g) {
  constexpr int NW = WM * WN;
  constexpr int NT = NW * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // per-wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_INS = BM / 8 / NW;  // glds wave-instructions per stage per wave
  constexpr int B_INS = BN / 8 / NW;
  static_assert(A_INS * 8 * NW == BM && B_INS * 8 * NW == BN, "tile / wave split");
  constexpr int STAGE = (BM + BN) * BK;  // fp16 elements per stage
  constexpr int LDS_ELEMS = S * STAGE > BM * (BN + 8) ? S * STAGE : BM * (BN + 8);
  __shared__ __attribute__((aligned(1024))) f16 lds[LDS_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wave_m = wid / WN, wave_n = wid % WN;

  // XCD-aware bijective remap (cdna_hip_programming.md §5 'XCD swizzle must be bijective'):
  // consecutive tile ids (same A row panel) land on one XCD's L2
  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  const int m0 = (wgid / tiles_n) * BM;
  const int n0 = (wgid % tiles_n) * BN;

  // per-lane glds sources: instruction i of this wave covers tile rows (wid*A_INS + i)*8 + lane/8
  const int lrow = lane >> 3;
  const int lchunk = (lane & 7) ^ lrow;  // pre-swizzled source chunk (row & 7 == lrow)
  const f16* a_src[A_INS];
  const f16* b_src[B_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) {
    int row = m0 + (wid * A_INS + i) * 8 + lrow;
    row = row < g.M ? row : g.M - 1;
    a_src[i] = g.A + (int64_t)row * g.lda + lchunk * 8;
  }
#pragma unroll
  for (int i = 0; i < B_INS; ++i) {
    int row = n0 + (wid * B_INS + i) * 8 + lrow;
    row = row < g.N ? row : g.N - 1;
    b_src[i] = g.B + (int64_t)row * g.ldb + lchunk * 8;
  }
  auto stage = [&](int buf, int k0) {
    f16* la = lds + buf * STAGE;
    f16* lb = la + BM * BK;
#pragma unroll
    for (int i = 0; i < A_INS; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(a_src[i] + k0),
                                       (lds_ptr_t)(la + (wid * A_INS + i) * 8 * BK), 16, 0, 0);
#pragma unroll
    for (int i = 0; i < B_INS; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b_src[i] + k0),
                                       (lds_ptr_t)(lb + (wid * B_INS + i) * 8 * BK), 16, 0, 0);
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int nk = g.K / BK;
  // prologue: S-1 stages in flight
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) stage(p, p * BK);

  const int fr = lane & 15, fg = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    // stage kt landed (this wave's DMA: leave the younger stages in flight), then one barrier:
    // every wave's DMA for kt is visible and every wave is done reading stage kt-1's buffer
    const int younger = min(S - 2, nk - 1 - kt);
    if constexpr (S >= 3) {
      if (younger >= 2) wait_vmcnt<2 * (A_INS + B_INS)>();
      else if (younger == 1) wait_vmcnt<A_INS + B_INS>();
      else wait_vmcnt<0>();
    } else {
      wait_vmcnt<0>();
    }
    __builtin_amdgcn_s_barrier();
    if (kt + S - 1 < nk) stage((kt + S - 1) % S, (kt + S - 1) * BK);
    const f16* la = lds + (kt % S) * STAGE;
    const f16* lb = la + BM * BK;
    // fragments of sub-step 1 are read while the MFMAs of sub-step 0 run (register double buffer)
    f16x8 af[2][TM], bf[2][TN];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wave_m * WTM + i * 16 + fr;
        af[s][i] = *(const f16x8*)(la + row * BK + swz(row, 4 * s + fg) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wave_n * WTN + j * 16 + fr;
        bf[s][j] = *(const f16x8*)(lb + row * BK + swz(row, 4 * s + fg) * 8);
      }
    }
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[s][j], af[s][i], acc[i][j], 0, 0, 0);
    if constexpr (PRIO) __builtin_amdgcn_s_setprio(0);
  }

  // epilogue.  lane holds C[m = .. + fr][n = .. + 4*fg + e], e = 0..3.
  if constexpr (EPI == EPI_F32) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wave_m * WTM + i * 16 + fr;
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + wave_n * WTN + j * 16 + 4 * fg;
        if (n < g.N) *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = acc[i][j];
      }
    }
  } else {
    // 1) the first fp16 rounding point in registers (fp16(acc + bias) / fp16(acc)), staged through LDS
    //    as a [BM][BN+8] fp16 tile; 2) the whole workgroup streams rows out with 16-byte accesses
    //    (full cache lines) applying the rest of the epilogue (residual, QuickGELU, QuickGELU').
    constexpr int LDC = BN + 8;
    f16* sC = lds;
    __syncthreads();  // every wave is done with the operand ring
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = wave_m * WTM + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = wave_n * WTN + j * 16 + 4 * fg;
        f32x4 v = acc[i][j];
        f16x4 t;
        if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU) {
          const int n = min(n0 + nl, g.N - 4);
          f16x4 b = *(const f16x4*)(g.bias + n);
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (f16)(v[e] + (float)b[e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (f16)v[e];
        }
        *(f16x4*)(sC + ml * LDC + nl) = t;
      }
    }
    __syncthreads();
    constexpr int CPR = BN / 8;        // 16-byte chunks per tile row
    constexpr int RPP = NT / CPR;      // rows per pass
    const int c8 = tid % CPR;
    const int n = n0 + 8 * c8;
    const int cnt = min(8, g.N - n);
    if (cnt > 0) {
#pragma unroll 4
      for (int r = tid / CPR; r < BM; r += RPP) {
        const int m = m0 + r;
        if (m < g.M) epi8<EPI>(g, m, n, cnt, sC + r * LDC + 8 * c8);
      }
    }
  }
}

template <int BM, int BN, int WM, int WN, int S>
int launch_tile(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles), block(WM * WN * 64);
  switch (epi) {
    case EPI_NONE: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_NONE><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_BIAS><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RESID: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_BIAS_RESID><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_BIAS_GELU><<<grid, block, 0, st>>>(a); break;
    case EPI_DGELU: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_DGELU><<<grid, block, 0, st>>>(a); break;
    case EPI_F32: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_F32><<<grid, block, 0, st>>>(a); break;
    case EPI_RESID: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_RESID><<<grid, block, 0, st>>>(a); break;
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
  const int vec8 = (ldc % 8 == 0) && (ld_aux % 8 == 0) && ((uintptr_t)C % 16 == 0) &&
                   (!aux_in || (uintptr_t)aux_in % 16 == 0) && (!aux_out || (uintptr_t)aux_out % 16 == 0);
  GemmArgs a{(const f16*)A, (const f16*)B, C, (const f16*)bias, (const f16*)aux_in, (f16*)aux_out,
             lda, ldb, ldc, ld_aux, M, N, K, vec8};
  hipStream_t st = (hipStream_t)stream;
  if (tile == 0) {  // heuristic: fill the 256 CUs
    int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
    tile = t128 >= 512 ? 1 : (t128 >= 256 ? 2 : 3);  // measured: tests/diagnostics/gemm_bench.py
  }
  switch (tile) {
    case 1: return launch_tile<128, 128, 2, 2, 2>(a, epilogue, st);
    case 2: return launch_tile<128, 64, 2, 2, 2>(a, epilogue, st);
    case 3: return launch_tile<64, 64, 2, 2, 2>(a, epilogue, st);
    case 4: return launch_tile<256, 128, 4, 2, 2>(a, epilogue, st);
    case 5: return launch_tile<256, 128, 4, 2, 3>(a, epilogue, st);
    case 6: return launch_tile<128, 128, 2, 2, 3>(a, epilogue, st);
    case 7: return launch_tile<128, 64, 2, 2, 3>(a, epilogue, st);
    case 8: return launch_tile<128, 256, 2, 4, 3>(a, epilogue, st);
    case 9: return launch_tile<256, 256, 2, 4, 2>(a, epilogue, st);
    case 10: return launch_tile<256, 128, 2, 2, 3>(a, epilogue, st);
    case 11: return launch_tile<128, 128, 2, 2, 4>(a, epilogue, st);
    case 12: return launch_tile<256, 128, 2, 2, 2>(a, epilogue, st);
    case 13: return launch_tile<128, 256, 2, 2, 3>(a, epilogue, st);
    case 14: return launch_tile<128, 64, 2, 2, 4>(a, epilogue, st);
    default: return mf_set_error("mf_gemm_nt: bad tile id", -2);
  }
}
