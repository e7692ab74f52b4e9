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
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mf_common.h"

namespace {

enum Epi : int {
  EPI_NONE = 0,        // C = fp16(acc)
  EPI_BIAS = 1,        // C = fp16(acc + bias)
  EPI_BIAS_RESID = 2,  // C = fp16(R + fp16(acc + bias))        (R = aux_in, may alias C)
  EPI_BIAS_GELU = 3,   // F = fp16(acc + bias) -> aux_out (if not null: the backward's operand) ; C = QuickGELU16(F)
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
  int vec8;    // C / aux row strides are multiples of 8 elements -> 16-byte epilogue accesses
  int ksplit;  // > 0: split-K slice of ksplit (multiple of 64) per slice z, fp32 partial at C + z*M*ldc
  int xb;      // log2 of the N-range count of the XCD blocking (tile_of); 0: M-ranges only; split-K: 1 =
               // N-major positions inside a slice (split_tile_of)
};

// The QuickGELU pre-activation (EPI_BIAS_GELU's aux output) is read again only by the backward, so it is
// stored non-temporally: it streams past the L2, which keeps the operand panels of the running tiles
// (r02 same-box A/B, scripts/ab_gemm_dirs.sh: v.fc 661 -> 680 TFLOP/s isolated, the c4 step +1.2 %; the C
// outputs stay regular stores: their consumer launches next, and non-temporal C stores were step-neutral).
MF_DEV void st16_stream(f16* p, f16x8 v) { __builtin_nontemporal_store(v, (f16x8*)p); }

// Tile of position p (0 .. tiles_m*tiles_n-1) in the XCD-blocked order.  The bijective remap below gives
// each XCD a contiguous range of positions, and the positions enumerate 8 blocks, block x = M-range
// (x >> xb) of 8 >> xb  x  N-range (x & (2^xb - 1)) of 2^xb, each block's tiles M-major (N inner).  So an
// XCD's L2 holds one block: its A panels and B panels are each re-read by the tiles of the block only.
// With xb = 0 an XCD takes whole rows of tiles (every B panel: the full weight matrix); for products
// whose weight matrix exceeds an XCD's 4 MB L2 (N x K x 2 B at N = 3072, K = 768) splitting N too keeps
// the working set of the XCD's concurrently running tiles inside its L2 (the host picks xb).
MF_DEV void tile_of(int p, int tiles_m, int tiles_n, int xb, int& mt, int& nt) {
  const int nb = 1 << xb, ma = 8 >> xb;
  int off = 0;
#pragma unroll 1
  for (int x = 0; x < 8; ++x) {
    const int ia = x >> xb, jb = x & (nb - 1);
    const int m_lo = tiles_m * ia / ma, m_hi = tiles_m * (ia + 1) / ma;
    const int n_lo = tiles_n * jb / nb, n_hi = tiles_n * (jb + 1) / nb;
    const int sz = (m_hi - m_lo) * (n_hi - n_lo);
    if (p < off + sz) {
      const int loc = p - off, w = n_hi - n_lo;
      mt = m_lo + loc / w;
      nt = n_lo + loc % w;
      return;
    }
    off += sz;
  }
  mt = nt = 0;  // unreachable for p < tiles_m * tiles_n
}

// Split-K position p (0 .. splits*tiles-1): slice-major, so an XCD's contiguous range of positions is a
// run of one slice's tiles (and at most a piece of the next) and its L2 holds that slice's K-window of the
// few A and B panels the run touches, instead of every XCD reading every slice's panels (r02 PMC: the
// block-11 weight gradients read 163 MB per launch against 49 MB of operands with the slice in
// blockIdx.z).  Inside a slice the run goes along the longer tile dimension (n_major: M inner).
MF_DEV void split_tile_of(int p, int tiles_m, int tiles_n, bool n_major, int& z, int& mt, int& nt) {
  const int tiles = tiles_m * tiles_n;
  z = p / tiles;
  const int q = p - z * tiles;
  if (n_major) {
    nt = q / tiles_m;
    mt = q - nt * tiles_m;
  } else {
    mt = q / tiles_n;
    nt = q - mt * tiles_n;
  }
}

// Elementwise epilogue on 8 consecutive columns (fp16 staged value t = the GEMM result rounded at
// the reference's first rounding point: fp16(acc + bias) or fp16(acc)).  The global operand an
// epilogue reads (residual R or pre-activation F) is fetched by epi_prefetch BEFORE the LDS
// staging pass so its latency overlaps the staging; epi8 finishes with it.
template <int EPI>
constexpr bool epi_reads_aux() { return EPI == EPI_BIAS_RESID || EPI == EPI_RESID || EPI == EPI_DGELU; }

template <int EPI>
MF_DEV f16x8 epi_prefetch(const GemmArgs& g, int64_t m, int n, int cnt) {
  f16x8 v = {};
  if constexpr (epi_reads_aux<EPI>())
    if (cnt == 8 && g.vec8) v = *(const f16x8*)(g.aux_in + m * g.ld_aux + n);
  return v;
}

template <int EPI>
MF_DEV void epi8(const GemmArgs& g, int64_t m, int n, int cnt, const f16* t, f16x8 aux) {
  f16* crow = (f16*)g.C + m * g.ldc + n;
  if (cnt == 8 && g.vec8) {
    f16x8 tv = *(const f16x8*)t;
    f16x8 out;
    if constexpr (EPI == EPI_NONE || EPI == EPI_BIAS) {
      out = tv;
    } else if constexpr (EPI == EPI_BIAS_RESID || EPI == EPI_RESID) {
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = (f16)((float)aux[e] + (float)tv[e]);
    } else if constexpr (EPI == EPI_BIAS_GELU) {
      if (g.aux_out) st16_stream(g.aux_out + m * g.ld_aux + n, tv);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t2;
        out[e] = (f16)quick_gelu16((float)tv[e], &t2);
      }
    } else if constexpr (EPI == EPI_DGELU) {
#pragma unroll
      for (int e = 0; e < 8; ++e) out[e] = (f16)quick_gelu16_bwd((float)tv[e], (float)aux[e]);
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
      if (g.aux_out) g.aux_out[m * g.ld_aux + n + e] = (f16)tvv;
      o = quick_gelu16(tvv, &t2);
    } else if constexpr (EPI == EPI_DGELU) {
      o = quick_gelu16_bwd(tvv, (float)g.aux_in[m * g.ld_aux + n + e]);
    }
    crow[e] = (f16)o;
  }
}

constexpr int BK = 64;

// In-kernel timeline stamps for diagnostics (tests/diagnostics/gemm_stamps.cpp builds this file
// with MF_GEMM_STAMPS defined); compiled out of libmapfed.so.
#ifdef MF_GEMM_STAMPS
__device__ unsigned long long* g_stamps;
#define MF_STAMP(slot)                                                                             \
  do {                                                                                             \
    if (threadIdx.x == 0) {                                                                        \
      unsigned long long t_ = __builtin_amdgcn_s_memrealtime();                                    \
      g_stamps[(size_t)blockIdx.x * 8 + (slot)] = t_;                                              \
      if ((slot) == 0) {                                                                           \
        unsigned xcc_ = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));                     \
        unsigned hw_ = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));                      \
        g_stamps[(size_t)blockIdx.x * 8 + 6] = xcc_;                                               \
        g_stamps[(size_t)blockIdx.x * 8 + 7] = hw_;                                                \
      }                                                                                            \
    }                                                                                              \
  } while (0)
#else
#define MF_STAMP(slot) \
  do {                 \
  } while (0)
#endif

MF_DEV int swz(int row, int chunk) { return chunk ^ (row & 7); }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// Raw s_barrier that also stops the compiler from moving LDS accesses across it (the builtin alone
// carries no memory semantics); unlike __syncthreads() it emits no vmcnt(0), so LDS-DMA stays in
// flight across it.
MF_DEV void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// s_waitcnt vmcnt(n) lgkmcnt(0): LDS-DMA of all but the n youngest VMEM ops landed AND every ds_read
// of this wave completed (a buffer's readers are done before the barrier that follows)
template <int N>
MF_DEV void wait_vm_lgkm0() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (0 << 8) | ((N >> 4) << 14));
}

// s_waitcnt vmcnt(n) (gfx9 encoding: vmcnt[3:0] | expcnt[6:4]=7 | lgkmcnt[11:8]=15 | vmcnt[5:4]<<14)
template <int N>
MF_DEV void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt");
  __builtin_amdgcn_s_waitcnt((N & 15) | (7 << 4) | (15 << 8) | ((N >> 4) << 14));
}

// Epilogue shared by both kernel families: the first fp16 rounding point in registers
// (fp16(acc + bias) / fp16(acc)) staged through LDS as a [BM][BN+8] fp16 tile, then the whole
// workgroup streams rows out with 16-byte accesses (full cache lines) applying the rest of the
// epilogue (residual, QuickGELU, QuickGELU').  acc[i][j] holds C[m0 + mbase + i*16 + fr]
// [n0 + nbase + j*16 + 4*fg + e], e = 0..3.  The caller has barriered the operand ring.
template <int BM, int BN, int NT, int TM, int TN, int EPI>
MF_DEV void epilogue_store(const GemmArgs& g, f16* lds, const f32x4 (&acc)[TM][TN], int m0, int n0, int mbase,
                           int nbase, int tid, int fr, int fg) {
  if constexpr (EPI == EPI_F32) {
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + mbase + i * 16 + fr;
      if (m >= g.M) continue;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int n = n0 + nbase + j * 16 + 4 * fg;
        if (n < g.N) *(f32x4*)((float*)g.C + (int64_t)m * g.ldc + n) = acc[i][j];
      }
    }
  } else {
    constexpr int LDC = BN + 8;
    constexpr int CPR = BN / 8;    // 16-byte chunks per tile row
    constexpr int RPP = NT / CPR;  // rows per pass
    constexpr int NPASS = (BM + RPP - 1) / RPP;
    f16* sC = lds;
    const int c8 = tid % CPR;
    const int n = n0 + 8 * c8;
    const int cnt = min(8, g.N - n);
    const int r0 = tid / CPR;
    const bool st_ok = r0 < RPP;  // CPR not dividing NT (BN = 192): the leftover threads store nothing
    // global operands first: residual / pre-activation rows of this thread's store passes, bias
    f16x8 auxv[NPASS];
#pragma unroll
    for (int p = 0; p < NPASS; ++p) {
      const int m = m0 + r0 + p * RPP;
      auxv[p] = (st_ok && cnt > 0 && r0 + p * RPP < BM && m < g.M) ? epi_prefetch<EPI>(g, m, n, cnt) : f16x8{};
    }
    f16x4 bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU)
        bv[j] = *(const f16x4*)(g.bias + min(n0 + nbase + j * 16 + 4 * fg, g.N - 4));
      else
        bv[j] = f16x4{};
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int ml = mbase + i * 16 + fr;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int nl = nbase + j * 16 + 4 * fg;
        f32x4 v = acc[i][j];
        f16x4 t;
        if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU) {
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (f16)(v[e] + (float)bv[j][e]);
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) t[e] = (f16)v[e];
        }
        *(f16x4*)(sC + ml * LDC + nl) = t;
      }
    }
    __syncthreads();
    if (st_ok && cnt > 0) {
#pragma unroll
      for (int p = 0; p < NPASS; ++p) {
        const int r = r0 + p * RPP;
        const int m = m0 + r;
        if (r < BM && m < g.M) epi8<EPI>(g, m, n, cnt, sC + r * LDC + 8 * c8, auxv[p]);
      }
    }
  }
}

// Tile BM x BN, (WM x WN) waves each owning a (BM/WM) x (BN/WN) block of 16x16 MFMA tiles, BK = 64.
// Operands go HBM -> LDS by LDS-DMA (buffer_load ... lds, 16 B per lane, no VGPR round trip) through
// buffer descriptors sized to the operand, so rows past M / N (and, for K-major operands, k-rows
// past K) read as zero: no clamping and no K padding.  Two layouts per operand:
//   * row-major [rows][K] (TA/TB false, nn.Linear weights, activations): each wave instruction fills
//     8 rows x 128 B of a [rows][64] image whose 16-B chunk c of row r holds chunk c ^ (r & 7);
//     fragments by ds_read_b128;
//   * K-major [K][rows] (TA/TB true: dY^T / X of the weight gradients, W as [in] x [out] of the dX
//     products): each instruction fills 512/R k-rows x 2R bytes of a [64][R] image whose 16-B chunk c
//     of k-row k holds chunk c ^ fT(k); fragments by two ds_read_b64_tr_b16 (4 k each, hardware
//     transpose), conflict-free (bank model in the commit history of this file).
// The swizzles are applied to the per-lane SOURCE address (the LDS side of an LDS-DMA is lane-linear).
// Two LDS buffers: the loads of K-step t+1 are issued before the fragment reads + MFMAs of step t and
// drained by one vmcnt(0) + barrier per step (cdna_hip_programming.md §5.5 T3/T4 minimum 2-phase form).
template <int R>
MF_DEV int swz_t(int k) {  // 16-byte-chunk XOR of a K-major image with R fp16 per k-row
  if constexpr (R == 128) return 2 * ((k & 3) | (((k >> 3) & 1) << 2));
  else return 2 * (((k >> 1) & 1) | (((k >> 3) & 1) << 1));
}

// 16 k-values (k0 .. k0+7 of column c) of a K-major [64][R] image as one MFMA fragment
template <int R>
MF_DEV f16x8 frag_t(const f16* img, int kr0, int c0, int fr) {
  f16x4 h[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int k = kr0 + 4 * u + (fr >> 2);
    const int col = c0 + 4 * (fr & 3);
    const f16* p = img + k * R + ((((col >> 3) ^ swz_t<R>(k))) << 3) + (col & 7);
    s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
    h[u] = __builtin_bit_cast(f16x4, v);
  }
  return (f16x8){h[0][0], h[0][1], h[0][2], h[0][3], h[1][0], h[1][1], h[1][2], h[1][3]};
}

// LDS-DMA source offset (bytes, k0 = 0) of this lane's 16 B for wave instruction ins_i, and the
// instruction's element offset in the operand image: row-major [rows][64] or K-major [64][RW]
template <bool T, int RW>
MF_DEV void dma_setup(int lane, int wid, int64_t ld, int row0, int ins_i, int nins, int& voff, int& dst) {
  if constexpr (!T) {
    const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
    const int brow = (wid * nins + ins_i) * 8;
    voff = (int)((((int64_t)(row0 + brow + lrow)) * ld + lchunk * 8) * 2);
    dst = brow * BK;
  } else {
    constexpr int CPR = RW / 8;   // 16-B chunks per k-row
    constexpr int KR = 512 / RW;  // k-rows per instruction
    const int kbase = (wid * nins + ins_i) * KR;
    const int kr = kbase + lane / CPR;
    const int c = (lane % CPR) ^ swz_t<RW>(kr);
    voff = (int)(((int64_t)kr * ld + row0 + c * 8) * 2);
    dst = kbase * RW;
  }
}

// issue one stage's LDS-DMA (all offsets in the range-checked VGPR offset).  The buffer descriptors
// are built here from (pointer, byte range): a descriptor-typed parameter fails template
// substitution in hipcc's host pass, which silently drops the kernel's host stub.
template <int A_INS, int B_INS>
MF_DEV void dma_stage(const f16* A, int a_bytes, const f16* B, int b_bytes, f16* la, f16* lb,
                      const int* a_voff, const int* a_dst, const int* b_voff, const int* b_dst, int a_k, int b_k) {
  const auto a_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)A, 0, a_bytes, 0x00020000);
  const auto b_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)B, 0, b_bytes, 0x00020000);
#pragma unroll
  for (int i = 0; i < A_INS; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr_t)(la + a_dst[i]), 16, a_voff[i] + a_k, 0, 0, 0);
#pragma unroll
  for (int i = 0; i < B_INS; ++i)
    __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr_t)(lb + b_dst[i]), 16, b_voff[i] + b_k, 0, 0, 0);
}

template <int BM, int BN, int WM, int WN, int S, int EPI, bool TA = false, bool TB = false>
__global__ __launch_bounds__(WM * WN * 64) void gemm_nt_kernel(GemmArgs g0) {
  GemmArgs g = g0;
  constexpr int NW = WM * WN;
  constexpr int NT = NW * 64;
  constexpr int WTM = BM / WM, WTN = BN / WN;  // per-wave tile
  constexpr int TM = WTM / 16, TN = WTN / 16;
  constexpr int A_INS = BM / 8 / NW;  // LDS-DMA wave-instructions per stage per wave (1 KiB each)
  constexpr int B_INS = BN / 8 / NW;
  static_assert(A_INS * 8 * NW == BM && B_INS * 8 * NW == BN, "tile / wave split");
  static_assert((!TA || BM == 64 || BM == 128) && (!TB || BN == 64 || BN == 128), "K-major image widths");
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
  const int tiles_m = (g.M + BM - 1) / BM;
  // split-K with xb = 2: the r02 order (A/B baseline): slice = dispatch id / tiles, remap inside the slice
  const bool legacy = g.ksplit > 0 && g.xb == 2;
  const int nwg = legacy ? tiles_m * tiles_n : gridDim.x;
  const int bid = legacy ? blockIdx.x % nwg : blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int mt, nt;
  if (g.ksplit > 0) {  // split-K: this workgroup's K slice and partial-sum plane (EPI_F32)
    int z;
    if (legacy) {
      z = blockIdx.x / nwg;
      tile_of(wgid, tiles_m, tiles_n, 0, mt, nt);
    } else {
      split_tile_of(wgid, tiles_m, tiles_n, g.xb != 0, z, mt, nt);
    }
    const int k0 = z * g.ksplit;
    g.A += (int64_t)k0 * (TA ? g.lda : 1);
    g.B += (int64_t)k0 * (TB ? g.ldb : 1);
    g.K = min(g.ksplit, g.K - k0);
    g.C = (float*)g.C + (int64_t)z * g.M * g.ldc;
  } else {
    tile_of(wgid, tiles_m, tiles_n, g.xb, mt, nt);
  }
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // per-operand LDS-DMA: byte offset of this lane's 16 B for instruction i at k0 = 0 (all offsets in
  // the VGPR offset: the descriptor's range check covers it), and the instruction's LDS destination
  const int a_bytes = (int)((TA ? (int64_t)(g.K - 1) * g.lda + g.M : (int64_t)(g.M - 1) * g.lda + g.K) * 2);
  const int b_bytes = (int)((TB ? (int64_t)(g.K - 1) * g.ldb + g.N : (int64_t)(g.N - 1) * g.ldb + g.K) * 2);
  int a_voff[A_INS], a_dst[A_INS], b_voff[B_INS], b_dst[B_INS];
#pragma unroll
  for (int i = 0; i < A_INS; ++i) dma_setup<TA, BM>(lane, wid, g.lda, m0, i, A_INS, a_voff[i], a_dst[i]);
#pragma unroll
  for (int i = 0; i < B_INS; ++i) dma_setup<TB, BN>(lane, wid, g.ldb, n0, i, B_INS, b_voff[i], b_dst[i]);
  // K step k0 advances a row-major operand by k0 elements, a K-major one by k0 k-rows
  const int a_kstep = TA ? (int)(g.lda * 2) : 2, b_kstep = TB ? (int)(g.ldb * 2) : 2;
#define MF_STAGE(buf, k0)                                                                                     \
  dma_stage<A_INS, B_INS>(g.A, a_bytes, g.B, b_bytes, lds + (buf)*STAGE, lds + (buf)*STAGE + BM * BK, a_voff, a_dst, \
                          b_voff, b_dst, (k0)*a_kstep, (k0)*b_kstep)



  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  MF_STAMP(0);
  const int nk = (g.K + BK - 1) / BK;  // a ragged last K step only with both operands K-major (zero-filled)
  // prologue: S-1 stages in flight
#pragma unroll
  for (int p = 0; p < S - 1; ++p)
    if (p < nk) MF_STAGE(p, p * BK);

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
    if (kt == 0) MF_STAMP(1);
    if (kt + S - 1 < nk) MF_STAGE((kt + S - 1) % S, (kt + S - 1) * BK);
    const f16* la = lds + (kt % S) * STAGE;
    const f16* lb = la + BM * BK;
    // fragments of sub-step 1 are read while the MFMAs of sub-step 0 run (register double buffer)
    f16x8 af[2][TM], bf[2][TN];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int row = wave_m * WTM + i * 16 + fr;
        if constexpr (TA)
          af[s][i] = frag_t<BM>(la, 32 * s + 8 * fg, wave_m * WTM + i * 16, fr);
        else
          af[s][i] = *(const f16x8*)(la + row * BK + swz(row, 4 * s + fg) * 8);
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int row = wave_n * WTN + j * 16 + fr;
        if constexpr (TB)
          bf[s][j] = frag_t<BN>(lb, 32 * s + 8 * fg, wave_n * WTN + j * 16, fr);
        else
          bf[s][j] = *(const f16x8*)(lb + row * BK + swz(row, 4 * s + fg) * 8);
      }
    }
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[s][j], af[s][i], acc[i][j], 0, 0, 0);
  }

#undef MF_STAGE
  // epilogue.  lane holds C[m = .. + fr][n = .. + 4*fg + e], e = 0..3.
  MF_STAMP(2);
  __syncthreads();  // every wave is done with the operand ring
  epilogue_store<BM, BN, NT, TM, TN, EPI>(g, lds, acc, m0, n0, wave_m * WTM, wave_n * WTN, tid, fr, fg);
  MF_STAMP(3);
}

// ------------------------------------------------------------------------------------------------
// gemm8: 8 waves (512 threads), BM x BN tile with BM = 256 (or 128), one workgroup per CU.
// Why this shape: a CU pulls operands from L2 at roughly 64-70 GB/s (MI355X_MICROARCH.md, LDS gather
// rates), so the tile's FLOP per fetched byte sets the MFMA ceiling: 128x128 needs ~150 GB/s per CU
// at full MFMA rate (measured main loop 45-50 % of peak), 256x256 needs ~75 GB/s.
// Pipeline (cdna_hip_programming.md §5 T3+T4, restated for this kernel): a K-tile (BK = 64) is four
// phases (m-half, k-sub) in the order (0,0) (1,0) (1,1) (0,1); a phase issues the ds_reads of the
// NEXT phase's fragments (from data retired by an earlier barrier) ahead of its own MFMAs, so LDS
// latency hides under the matrix pipe.  The operands of a K-tile are four half-tiles
// [A k0, B k0, A k1, B k1] (sequence number 4*kt + h), each a [rows][32] fp16 image (64-byte rows,
// 16-byte chunk c of row r stored at c ^ ((-(r >> 2)) & 3): conflict-free ds_read_b128 fragment
// reads, checked with the bank model).  They live in a ring of NSLOT = 10 slots of SLOT bytes
// (160 KiB) and are filled by LDS-DMA (buffer_load ... lds, 16 rows x 64 B per wave instruction,
// swizzle applied to the source) TWO K-tiles ahead, one half-tile per phase: ~8 phases of latency
// cover before a counted vmcnt + barrier retires a pair (two such points per K-tile).  WAR: the
// half-tile a load overwrites (sequence - 10) was last read at least one barrier earlier and every
// ds_read completes (lgkmcnt(0)) before the next barrier.  A/B fragment register sets alternate
// statically (no copies, no scratch); the loop is peeled so the steady-state body has no branches.
template <int BM, int BN, int WM, int WN, int EPI>
__global__ __launch_bounds__(512) void gemm8_kernel(GemmArgs g) {
  constexpr int NT = 512;
  static_assert(WM * WN == 8, "8 waves");
  constexpr int WTM = BM / WM, WTN = BN / WN;
  constexpr int QM = WTM / 2;
  constexpr int QTM = QM / 16, TN = WTN / 16, TM = 2 * QTM;
  static_assert(QTM >= 1 && TN >= 1 && QM % 16 == 0, "phase shape");
  constexpr int A_INS = BM / 128;  // LDS-DMA wave instructions per wave per half-tile (rows x 64 B)
  constexpr int B_INS = BN / 128;
  static_assert(A_INS * 128 == BM && B_INS * 128 == BN, "half-tile split");
  constexpr int HK = 32;                                // k-sub width (elements)
  constexpr int SLOT = (BM > BN ? BM : BN) * HK;        // fp16 elements per ring slot
  constexpr int NSLOT = 10;
  constexpr int LDC = BN + 8;
  constexpr int LDS_ELEMS = NSLOT * SLOT > BM * LDC ? NSLOT * SLOT : BM * LDC;
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) f16 lds[LDS_ELEMS];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int mt, nt;
  tile_of(wgid, (g.M + BM - 1) / BM, tiles_n, g.xb, mt, nt);
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // LDS-DMA: instruction covers 16 rows x 64 B; lane l -> row (l >> 2), chunk (l & 3), whose source
  // chunk is pre-swizzled; rows past M (N) read as zero through the buffer descriptor's range (every
  // offset is in the range-checked VGPR offset, none in the scalar offset).
  const int src_chunk = (lane & 3) ^ ((-(lane >> 4)) & 3);
  const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, 0, (int)(((int64_t)(g.M - 1) * g.lda + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.B, 0, (int)(((int64_t)(g.N - 1) * g.ldb + g.K) * 2), 0x00020000);
  const int a_voff = ((lane >> 2) * (int)g.lda + src_chunk * 8) * 2;
  const int b_voff = ((lane >> 2) * (int)g.ldb + src_chunk * 8) * 2;
  auto slot = [&](int seq) { return lds + (seq % NSLOT) * SLOT; };
  // issue half-tile h (0: A k0, 1: B k0, 2: A k1, 3: B k1) of K-tile kt
  auto issue = [&](int kt, int h) {
    f16* dst = slot(4 * kt + h);
    const int kofs = kt * BK + HK * (h >> 1);
    if ((h & 1) == 0) {
#pragma unroll
      for (int i = 0; i < A_INS; ++i) {
        const int row = (wid * A_INS + i) * 16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr_t)(dst + row * HK), 16,
                                                 a_voff + (int)(((int64_t)(m0 + row) * g.lda + kofs) * 2), 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < B_INS; ++i) {
        const int row = (wid * B_INS + i) * 16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr_t)(dst + row * HK), 16,
                                                 b_voff + (int)(((int64_t)(n0 + row) * g.ldb + kofs) * 2), 0, 0, 0);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fg = lane >> 4;
  // fragment (row, k 8*fg..8*fg+7 of the k-sub) of a [rows][32] image: row = base16 + fr
  const int frag_off = fr * HK + ((fg ^ ((-(fr >> 2)) & 3)) << 3);
  auto read_a = [&](f16x8 (&af)[QTM], const f16* img, int mh) {
#pragma unroll
    for (int i = 0; i < QTM; ++i) af[i] = *(const f16x8*)(img + (wm * WTM + mh * QM + i * 16) * HK + frag_off);
  };
  auto read_b = [&](f16x8 (&bf)[TN], const f16* img) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *(const f16x8*)(img + (wn * WTN + j * 16) * HK + frag_off);
  };
  auto mma = [&](const f16x8 (&af)[QTM], const f16x8 (&bf)[TN], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < QTM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[mh * QTM + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[mh * QTM + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = g.K / BK;  // >= 2 (the launcher routes K = 64 elsewhere)
  MF_STAMP(0);
  // prologue: K-tiles 0 and 1 (eight half-tiles); retire A k0, B k0 of K-tile 0 and read phase 0's
  // fragments A(0, k0), B(k0)
#pragma unroll
  for (int h = 0; h < 4; ++h) issue(0, h);
#pragma unroll
  for (int h = 0; h < 4; ++h) issue(1, h);
  f16x8 fx[QTM], fy[QTM], fb0[TN], fb1[TN];
  wait_vm_lgkm0<3 * A_INS + 3 * B_INS>();
  lds_barrier();
  read_a(fx, slot(0), 0);
  read_b(fb0, slot(1));
  MF_STAMP(1);

  // one K-tile.  MODE 0: steady state (issues K-tile kt+2);  MODE 1: kt = nk-2 (nothing left to
  // issue);  MODE 2: kt = nk-1 (the last).  The vmcnt of a retire point = wave instructions issued
  // after the retired pair.
  auto ktile = [&](int kt, auto mode_tag) {
    constexpr int MODE = decltype(mode_tag)::value;
    const f16* a0 = slot(4 * kt + 0);
    const f16* a1 = slot(4 * kt + 2);
    const f16* b1 = slot(4 * kt + 3);
    // phase 0 (m-half 0, k0): next reads A(1, k0)
    read_a(fy, a0, 1);
    if constexpr (MODE == 0) issue(kt + 2, 0);
    mma(fx, fb0, 0);
    // retire A k1, B k1 of this K-tile
    wait_vm_lgkm0<MODE == 0 ? 3 * A_INS + 2 * B_INS : (MODE == 1 ? 2 * A_INS + 2 * B_INS : 0)>();
    lds_barrier();
    // phase 1 (m-half 1, k0): next reads A(1, k1), B(k1)
    read_a(fx, a1, 1);
    read_b(fb1, b1);
    if constexpr (MODE == 0) issue(kt + 2, 1);
    mma(fy, fb0, 1);
    // phase 2 (m-half 1, k1): next reads A(0, k1)
    read_a(fy, a1, 0);
    if constexpr (MODE == 0) issue(kt + 2, 2);
    mma(fx, fb1, 1);
    if constexpr (MODE != 2) {
      // retire A k0, B k0 of the next K-tile
      wait_vm_lgkm0<MODE == 0 ? 3 * A_INS + 2 * B_INS : A_INS + B_INS>();
      lds_barrier();
      // phase 3 (m-half 0, k1): next reads A(0, k0), B(k0) of the next K-tile
      read_a(fx, slot(4 * kt + 4), 0);
      read_b(fb0, slot(4 * kt + 5));
      if constexpr (MODE == 0) issue(kt + 2, 3);
    }
    mma(fy, fb1, 0);
  };
  for (int kt = 0; kt < nk - 2; ++kt) ktile(kt, std::integral_constant<int, 0>{});
  ktile(nk - 2, std::integral_constant<int, 1>{});
  ktile(nk - 1, std::integral_constant<int, 2>{});
  MF_STAMP(2);

  __syncthreads();  // every wave is done with the operand ring (no DMA outstanding after the last K-tile)
  epilogue_store<BM, BN, NT, TM, TN, EPI>(g, lds, acc, m0, n0, wm * WTM, wn * WTN, tid, fr, fg);
  MF_STAMP(3);
}


// gemm8s: the 256x256 8-wave tile with the two wave rows (wm = 0, 1) staggered by one barrier (ping-pong,
// cdna_hip_programming.md §5 "The 256² 8-phase template"): every phase is a memory section (fragment
// ds_reads for this phase's MFMAs, one half-tile of LDS-DMA, the retire waits) and a compute section
// (16 MFMAs), separated by barriers; wave row 1 runs one barrier behind row 0, so on each SIMD one wave
// issues MFMAs while its partner loads.  Ring of 10 half-tile slots, half-tile H issued in the memory
// section of phase H - 7.  With the stagger (derivation in DESIGN.md §6):
//   RAW: a half-tile first read in phase f is retired (counted vmcnt) at the end of memory section f - 1;
//   WAR: a slot last read in phase q is refilled in phase q + 2 or later (H - 10 is last read in phase
//        <= H - 9, refilled in H - 7).
template <int EPI>
__global__ __launch_bounds__(512) void gemm8s_kernel(GemmArgs g) {
  constexpr int BM = 256, BN = 256, WM = 2, WN = 4, NT = 512;
  constexpr int WTM = BM / WM, WTN = BN / WN, QM = WTM / 2;
  constexpr int QTM = QM / 16, TN = WTN / 16, TM = 2 * QTM;
  constexpr int INS = 2;                 // LDS-DMA wave instructions per wave per half-tile (A and B alike)
  constexpr int HK = 32;
  constexpr int SLOT = 256 * HK;
  constexpr int NSLOT = 10, E = 7;
  constexpr int LDC = BN + 8;
  constexpr int LDS_ELEMS = NSLOT * SLOT > BM * LDC ? NSLOT * SLOT : BM * LDC;
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) f16 lds[LDS_ELEMS];

  MF_STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int mt, nt;
  tile_of(wgid, (g.M + BM - 1) / BM, tiles_n, g.xb, mt, nt);
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  const int src_chunk = (lane & 3) ^ ((-(lane >> 4)) & 3);
  const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, 0, (int)(((int64_t)(g.M - 1) * g.lda + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.B, 0, (int)(((int64_t)(g.N - 1) * g.ldb + g.K) * 2), 0x00020000);
  const int a_voff = ((lane >> 2) * (int)g.lda + src_chunk * 8) * 2;
  const int b_voff = ((lane >> 2) * (int)g.ldb + src_chunk * 8) * 2;
  auto slot = [&](int h) { return lds + (h % NSLOT) * SLOT; };
  // issue half-tile H (K-tile H / 4; 0: A k0, 1: B k0, 2: A k1, 3: B k1)
  auto issue = [&](int H) {
    f16* dst = slot(H);
    const int kofs = (H >> 2) * BK + HK * ((H >> 1) & 1);
    if ((H & 1) == 0) {
#pragma unroll
      for (int i = 0; i < INS; ++i) {
        const int row = (wid * INS + i) * 16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(a_rsrc, (lds_ptr_t)(dst + row * HK), 16,
                                                 a_voff + (int)(((int64_t)(m0 + row) * g.lda + kofs) * 2), 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < INS; ++i) {
        const int row = (wid * INS + i) * 16;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(b_rsrc, (lds_ptr_t)(dst + row * HK), 16,
                                                 b_voff + (int)(((int64_t)(n0 + row) * g.ldb + kofs) * 2), 0, 0, 0);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  const int frag_off = fr * HK + ((fg ^ ((-(fr >> 2)) & 3)) << 3);
  auto read_a = [&](f16x8 (&af)[QTM], const f16* img, int mh) {
#pragma unroll
    for (int i = 0; i < QTM; ++i) af[i] = *(const f16x8*)(img + (wm * WTM + mh * QM + i * 16) * HK + frag_off);
  };
  auto read_b = [&](f16x8 (&bf)[TN], const f16* img) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *(const f16x8*)(img + (wn * WTN + j * 16) * HK + frag_off);
  };
  auto mma = [&](const f16x8 (&af)[QTM], const f16x8 (&bf)[TN], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < QTM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[mh * QTM + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[mh * QTM + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = g.K / BK;  // >= 2
  const int nh = 4 * nk;
  // prologue: half-tiles 0 .. 6 (nk >= 2: 8 exist), retire 0 and 1 (first read in phase 0)
#pragma unroll
  for (int h = 0; h < E; ++h) issue(h);
  wait_vmcnt<INS * (E - 2)>();
  lds_barrier();
  MF_STAMP(1);
  if (wm == 1) lds_barrier();  // the stagger
  f16x8 fx[QTM], fy[QTM], fb0[TN], fb1[TN];

  // one K-tile; MODE 0: steady (issues half-tiles 4kt+7 .. 4kt+10), 1: kt = nk-2 (issues 4nk-1 only),
  // 2: kt = nk-1 (none).  Retire counts = INS x half-tiles issued after the retired ones.
  auto ktile = [&](int kt, auto mode_tag) {
    constexpr int MODE = decltype(mode_tag)::value;
    const int h0 = 4 * kt;
    // phase 0 (m-half 0, k-sub 0)
    read_a(fx, slot(h0), 0);
    read_b(fb0, slot(h0 + 1));
    if constexpr (MODE <= 1) issue(h0 + E);
    lds_barrier();
    mma(fx, fb0, 0);
    lds_barrier();
    // phase 1 (m-half 1, k-sub 0); retire half-tiles h0+2, h0+3 (first read in phase 2)
    read_a(fy, slot(h0), 1);
    if constexpr (MODE == 0) issue(h0 + E + 1);
    if constexpr (MODE == 0) wait_vmcnt<INS * 5>();
    else if constexpr (MODE == 1) wait_vmcnt<INS * 4>();
    else wait_vmcnt<0>();
    lds_barrier();
    mma(fy, fb0, 1);
    lds_barrier();
    // phase 2 (m-half 1, k-sub 1)
    read_a(fx, slot(h0 + 2), 1);
    read_b(fb1, slot(h0 + 3));
    if constexpr (MODE == 0) issue(h0 + E + 2);
    lds_barrier();
    mma(fx, fb1, 1);
    lds_barrier();
    // phase 3 (m-half 0, k-sub 1); retire half-tiles h0+4, h0+5 (first read in the next K-tile's phase 0)
    read_a(fy, slot(h0 + 2), 0);
    if constexpr (MODE == 0) issue(h0 + E + 3);
    if constexpr (MODE == 0) wait_vmcnt<INS * 5>();
    else if constexpr (MODE == 1) wait_vmcnt<INS * 2>();
    lds_barrier();
    mma(fy, fb1, 0);
    lds_barrier();
  };
  for (int kt = 0; kt < nk - 2; ++kt) ktile(kt, std::integral_constant<int, 0>{});
  ktile(nk - 2, std::integral_constant<int, 1>{});
  ktile(nk - 1, std::integral_constant<int, 2>{});
  (void)nh;
  if (wm == 0) lds_barrier();  // even out the barrier count
  __syncthreads();
  MF_STAMP(2);
  epilogue_store<BM, BN, NT, TM, TN, EPI>(g, lds, acc, m0, n0, wm * WTM, wn * WTN, tid, fr, fg);
  MF_STAMP(3);
}

// gemm8f: the 256x256 8-wave staggered tile of gemm8s with FULL-LINE operand images.  gemm8s stages
// [256 rows][32 k] half-tiles, so each LDS-DMA wave instruction covers 16 rows x 64 B: half of 16 cache lines,
// each line fetched twice per K-tile (once per k-sub) -- its TA address/command FIFOs run full 4x as often as
// hipBLASLt's (r04 PMC).  Here a half-tile is 128 rows x the whole K-tile ([128][64] fp16, 128-B rows, 16-B chunk
// c of row r at c ^ (r & 7): the 4-wave kernel's conflict-free image), so an instruction covers 8 whole lines
// (cdna_hip_programming.md §5 "The 256² 8-phase template": 128-row halves of A and B, BK = 64).  Half-tiles of
// K-tile t, in issue order: H = 4t + {0: B rows 0-127, 1: B rows 128-255, 2: A rows 0-127, 3: A rows 128-255};
// wave (wm, wn) reads A half wm and B half wn >> 1.  Phases (m-half, k-sub) as gemm8s, so every accumulator sums
// its k-subs in ascending order: bit-identical to gemm8s and to the 4-wave tiles.  Ring of NSLOT = 10 half-tile
// slots (160 KiB), half-tile H issued in the memory section of phase H - E (E = 6), K-tile t+1's four half-tiles
// retired (vmcnt(2 half-tiles), then the barrier) in the memory section of phase 4t + 3.  Hazards under the
// one-barrier stagger (row 1 runs a barrier behind row 0; row r's memory section of phase P lies between barrier
// instances 2P + r and 2P + r + 1, its reads complete before instance 2P + r + 2):
//   RAW: both rows' waits for K-tile t precede instance 8t, the first read of row 0 follows it;
//   WAR: B halves are last read in phase 4t + 2 (both rows), A0 in 4t + 3 (row 0), A1 in 4t + 3 (row 1); the slot
//        of H = 4t + h held H - 10 (h = 0, 1: A0 / A1 of t - 3; h = 2, 3: B0 / B1 of t - 2), refilled in phase
//        H - 6 >= (last read) + 2 in every case (h = 2 tight: B0 of t - 2 last read 4t - 6, refilled 4t - 4).
template <int EPI>
__global__ __launch_bounds__(512) void gemm8f_kernel(GemmArgs g) {
  constexpr int BM = 256, BN = 256, WN = 4, NT = 512;
  constexpr int WTM = 128, WTN = 64, QTM = 4, TN = 4, TM = 8;
  constexpr int HALF = 128 * BK;  // fp16 elements per half-tile image
  constexpr int NSLOT = 10, E = 6;
  constexpr int LDC = BN + 8;
  constexpr int LDS_ELEMS = NSLOT * HALF > BM * LDC ? NSLOT * HALF : BM * LDC;
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) f16 lds[LDS_ELEMS];

  MF_STAMP(0);
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_n = (g.N + BN - 1) / BN;
  const int nwg = gridDim.x;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wgid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  int mt, nt;
  tile_of(wgid, (g.M + BM - 1) / BM, tiles_n, g.xb, mt, nt);
  const int m0 = mt * BM;
  const int n0 = nt * BN;

  // LDS-DMA: a wave instruction fills 8 rows x 128 B; lane l -> row l >> 3, chunk (l & 7) whose source chunk is
  // pre-swizzled; wave w fills rows (2w + i) * 8 .. + 7 (i = 0, 1) of every half-tile
  const int lrow = lane >> 3, schunk = (lane & 7) ^ lrow;
  const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, 0, (int)(((int64_t)(g.M - 1) * g.lda + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.B, 0, (int)(((int64_t)(g.N - 1) * g.ldb + g.K) * 2), 0x00020000);
  const int a_voff = (lrow * (int)g.lda + schunk * 8) * 2;
  const int b_voff = (lrow * (int)g.ldb + schunk * 8) * 2;
  auto slot = [&](int h) { return lds + (h % NSLOT) * HALF; };
  auto issue = [&](int H) {
    f16* dst = slot(H);
    const int kofs = (H >> 2) * BK;
    const int hh = H & 3;
    if (hh < 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wid * 2 + i) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            b_rsrc, (lds_ptr_t)(dst + row * BK), 16,
            b_voff + (int)(((int64_t)(n0 + hh * 128 + row) * g.ldb + kofs) * 2), 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wid * 2 + i) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            a_rsrc, (lds_ptr_t)(dst + row * BK), 16,
            a_voff + (int)(((int64_t)(m0 + (hh - 2) * 128 + row) * g.lda + kofs) * 2), 0, 0, 0);
      }
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fg = lane >> 4;
  // fragment (row fr of a 16-row block, k 8fg .. 8fg + 7 of k-sub s) of a [128][64] image
  const int foff0 = fr * BK + ((fg ^ (fr & 7)) << 3);
  const int foff1 = fr * BK + (((4 + fg) ^ (fr & 7)) << 3);
  const int a_row0 = 0, b_row0 = (wn & 1) * WTN;
  auto read_a = [&](f16x8 (&af)[QTM], const f16* img, int mh, int foff) {
#pragma unroll
    for (int i = 0; i < QTM; ++i) af[i] = *(const f16x8*)(img + (a_row0 + mh * 64 + i * 16) * BK + foff);
  };
  auto read_b = [&](f16x8 (&bf)[TN], const f16* img, int foff) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *(const f16x8*)(img + (b_row0 + j * 16) * BK + foff);
  };
  auto mma = [&](const f16x8 (&af)[QTM], const f16x8 (&bf)[TN], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < QTM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[mh * QTM + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[mh * QTM + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };

  const int nk = g.K / BK;  // >= 2
  // prologue: half-tiles 0 .. 5; retire K-tile 0 (0 .. 3)
#pragma unroll
  for (int h = 0; h < E; ++h) issue(h);
  wait_vmcnt<2 * 2>();
  lds_barrier();
  MF_STAMP(1);
  if (wm == 1) lds_barrier();  // the stagger
  f16x8 fx[QTM], fy[QTM], fb0[TN], fb1[TN];

  // one K-tile; MODE 0: steady (issues 4t+6 .. 4t+9, retires K-tile t+1 with two half-tiles in flight),
  // 1: t = nk-2 (issues 4t+6, 4t+7 = the last two, retires K-tile t+1 with nothing in flight), 2: t = nk-1.
  auto ktile = [&](int kt, auto mode_tag) {
    constexpr int MODE = decltype(mode_tag)::value;
    const int h0 = 4 * kt;
    const f16* ia = slot(h0 + 2 + wm);
    const f16* ib = slot(h0 + (wn >> 1));
    // phase 0 (m-half 0, k-sub 0)
    read_a(fx, ia, 0, foff0);
    read_b(fb0, ib, foff0);
    if constexpr (MODE <= 1) issue(h0 + E);
    lds_barrier();
    mma(fx, fb0, 0);
    lds_barrier();
    // phase 1 (m-half 1, k-sub 0)
    read_a(fy, ia, 1, foff0);
    if constexpr (MODE <= 1) issue(h0 + E + 1);
    lds_barrier();
    mma(fy, fb0, 1);
    lds_barrier();
    // phase 2 (m-half 1, k-sub 1)
    read_a(fx, ia, 1, foff1);
    read_b(fb1, ib, foff1);
    if constexpr (MODE == 0) issue(h0 + E + 2);
    lds_barrier();
    mma(fx, fb1, 1);
    lds_barrier();
    // phase 3 (m-half 0, k-sub 1); retire the next K-tile
    read_a(fy, ia, 0, foff1);
    if constexpr (MODE == 0) {
      issue(h0 + E + 3);
      wait_vmcnt<2 * 2>();
    } else if constexpr (MODE == 1) {
      wait_vmcnt<0>();
    }
    lds_barrier();
    mma(fy, fb1, 0);
    lds_barrier();
  };
  for (int kt = 0; kt < nk - 2; ++kt) ktile(kt, std::integral_constant<int, 0>{});
  ktile(nk - 2, std::integral_constant<int, 1>{});
  ktile(nk - 1, std::integral_constant<int, 2>{});
  if (wm == 0) lds_barrier();  // even out the barrier count
  __syncthreads();
  MF_STAMP(2);
  epilogue_store<BM, BN, NT, TM, TN, EPI>(g, lds, acc, m0, n0, wm * WTM, wn * WTN, tid, fr, fg);
  MF_STAMP(3);
}

// gemm8p: gemm8f made persistent for launches of many rounds of 256x256 tiles (the eval engine's products at
// EVAL_GROUP 4, M = 79 600; the C5 text tower, M = 77 000).  In-kernel stamps of gemm8f on those launches
// (tests/diagnostics/gemm_stamps.cpp, profiles/r06_v6_gemm_stamps_eval4.txt): a 12-K-step tile lives ~29 us, of
// which the prologue (the first K-tile's DMA round trip) is ~4 us and the epilogue ~4-7 us, and a new workgroup
// starts ~3 us after its predecessor ends -- with one 160 KB workgroup per CU nothing else runs meanwhile.  Here one
// workgroup per CU walks its XCD's tiles (the positions tile_of gives the XCD), and where the epilogue reads no
// global operand (EPI_NONE / EPI_BIAS / EPI_BIAS_GELU) the NEXT tile's first six half-tiles are issued into the
// (by then free) ring before this tile's epilogue, whose results go straight from registers to buffer stores (no
// LDS staging; rows past M fall outside the buffer range and are dropped, so every wave issues the same count and
// the counted vmcnt stays exact).  Epilogues that read aux (residual, QuickGELU') run before the next prologue:
// a plain load while LDS-DMA is in flight would make the compiler drain it.  Main loop, fragment reads, MFMA
// order and the epilogue arithmetic are gemm8f's / epilogue_store's: bit-identical (tests/test_kernels_gpu.py).
// Needs N % 256 == 0, K % 64 == 0, fp16 C, 16-byte aligned C / aux with 8-element strides (the host checks).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// s_waitcnt lgkmcnt(0) alone (vmcnt 63 = no wait): this wave's ds_reads / ds_writes done, LDS-DMA left in flight
MF_DEV void wait_lgkm0() { __builtin_amdgcn_s_waitcnt((15) | (7 << 4) | (0 << 8) | (3 << 14)); }

// gemm8p's epilogue while the next tile's first six half-tiles fly into ring slots 0..5: the tile's two 128-row
// halves in turn staged through slots 6..9 ([128][256] fp16, 16-byte chunk c of row r at c ^ (r & 7)) by the four
// waves that own the half, then every thread streams 16-byte chunks out (full cache lines) through buffer stores
// (rows past M fall outside the range: dropped, so each thread issues exactly 8 stores per half, 8 more for the
// pre-activation).  The arithmetic is epilogue_store's: fp16(acc + bias), then epi8's QuickGELU.
template <int EPI>
MF_DEV void epilogue_staged8p(const GemmArgs& g, f16* stage, const f32x4 (&acc)[8][4], const f16x4 (&bv)[4], int m0,
                              int n0, int wm, int wn, int tid, int fr, int fg, __amdgpu_buffer_rsrc_t c_rsrc,
                              __amdgpu_buffer_rsrc_t x_rsrc) {
  static_assert(EPI == EPI_NONE || EPI == EPI_BIAS || EPI == EPI_BIAS_GELU, "epilogues without a global read");
#pragma unroll
  for (int hh = 0; hh < 2; ++hh) {
    if (wm == hh) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = i * 16 + fr;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int col = wn * 64 + j * 16 + 4 * fg;
          f16x4 t;
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) t[e] = (f16)(acc[i][j][e] + (float)bv[j][e]);
            else t[e] = (f16)acc[i][j][e];
          }
          *(f16x4*)(stage + r * 256 + ((((col >> 3) ^ (r & 7))) << 3) + (col & 7)) = t;
        }
      }
    }
    wait_lgkm0();
    lds_barrier();
#pragma unroll
    for (int pass = 0; pass < 8; ++pass) {
      const int r = pass * 16 + (tid >> 5), c = tid & 31;
      const f16x8 tv = *(const f16x8*)(stage + r * 256 + ((c ^ (r & 7)) << 3));
      const int m = m0 + hh * 128 + r, n = n0 + 8 * c;
      f16x8 out;
      if constexpr (EPI == EPI_NONE || EPI == EPI_BIAS) {
        out = tv;
      } else {
        if (g.aux_out)  // the pre-activation, non-temporal (st16_stream's policy)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, tv), x_rsrc,
                                                 (int)(((int64_t)m * g.ld_aux + n) * 2), 0, 2);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          float t2;
          out[e] = (f16)quick_gelu16((float)tv[e], &t2);
        }
      }
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, out), c_rsrc,
                                             (int)(((int64_t)m * g.ldc + n) * 2), 0, 0);
    }
    wait_lgkm0();
    lds_barrier();  // the staging area is read before the next half (or the next tile's DMA) overwrites it
  }
}

template <int EPI>
__global__ __launch_bounds__(512) void gemm8p_kernel(GemmArgs g) {
  constexpr int BM = 256, BN = 256, WN = 4;
  constexpr int WTM = 128, WTN = 64, QTM = 4, TN = 4, TM = 8;
  constexpr int HALF = 128 * BK;
  constexpr int NSLOT = 10, E = 6;
  static_assert(!epi_reads_aux<EPI>(), "epilogues that read a global operand stay on gemm8f");
  static_assert(NSLOT * HALF * 2 <= 160 * 1024 && BM * (BN + 8) <= NSLOT * HALF && 128 * 256 <= 4 * HALF, "LDS");
  __shared__ __attribute__((aligned(1024))) f16 lds[NSLOT * HALF];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;
  const int tiles_m = (g.M + BM - 1) / BM, tiles_n = g.N / BN;
  const int T = tiles_m * tiles_n;
  // this workgroup's positions: XCD x's contiguous range (the bijective remap of the one-shot kernels), every
  // nl-th position from l
  const int x = blockIdx.x & 7, l = blockIdx.x >> 3, nl = gridDim.x >> 3;
  const int q8 = T >> 3, r8 = T & 7;
  const int pstart = x < r8 ? x * (q8 + 1) : r8 * (q8 + 1) + (x - r8) * q8;
  const int psize = q8 + (x < r8 ? 1 : 0);
  int k = l;
  if (k >= psize) return;  // whole workgroup

  const int lrow = lane >> 3, schunk = (lane & 7) ^ lrow;
  const __amdgpu_buffer_rsrc_t a_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.A, 0, (int)(((int64_t)(g.M - 1) * g.lda + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t b_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)g.B, 0, (int)(((int64_t)(g.N - 1) * g.ldb + g.K) * 2), 0x00020000);
  const __amdgpu_buffer_rsrc_t c_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      g.C, 0, (int)(((int64_t)(g.M - 1) * g.ldc + g.N) * 2), 0x00020000);
  const void* xptr = (const void*)g.aux_out;
  const __amdgpu_buffer_rsrc_t x_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      (void*)xptr, 0, xptr ? (int)(((int64_t)(g.M - 1) * g.ld_aux + g.N) * 2) : 0, 0x00020000);
  const int a_voff = (lrow * (int)g.lda + schunk * 8) * 2;
  const int b_voff = (lrow * (int)g.ldb + schunk * 8) * 2;
  auto slot = [&](int h) { return lds + (h % NSLOT) * HALF; };
  int m0, n0;
  auto tile_at = [&](int kk, int& mm0, int& nn0) {
    int mt, nt;
    tile_of(pstart + kk, tiles_m, tiles_n, g.xb, mt, nt);
    mm0 = mt * BM;
    nn0 = nt * BN;
  };
  auto issue = [&](int H, int mm0, int nn0) {
    f16* dst = slot(H);
    const int kofs = (H >> 2) * BK;
    const int hh = H & 3;
    if (hh < 2) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wid * 2 + i) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            b_rsrc, (lds_ptr_t)(dst + row * BK), 16,
            b_voff + (int)(((int64_t)(nn0 + hh * 128 + row) * g.ldb + kofs) * 2), 0, 0, 0);
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int row = (wid * 2 + i) * 8;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            a_rsrc, (lds_ptr_t)(dst + row * BK), 16,
            a_voff + (int)(((int64_t)(mm0 + (hh - 2) * 128 + row) * g.lda + kofs) * 2), 0, 0, 0);
      }
    }
  };

  f32x4 acc[TM][TN];
  const int fr = lane & 15, fg = lane >> 4;
  const int foff0 = fr * BK + ((fg ^ (fr & 7)) << 3);
  const int foff1 = fr * BK + (((4 + fg) ^ (fr & 7)) << 3);
  const int a_row0 = 0, b_row0 = (wn & 1) * WTN;
  auto read_a = [&](f16x8 (&af)[QTM], const f16* img, int mh, int foff) {
#pragma unroll
    for (int i = 0; i < QTM; ++i) af[i] = *(const f16x8*)(img + (a_row0 + mh * 64 + i * 16) * BK + foff);
  };
  auto read_b = [&](f16x8 (&bf)[TN], const f16* img, int foff) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bf[j] = *(const f16x8*)(img + (b_row0 + j * 16) * BK + foff);
  };
  auto mma = [&](const f16x8 (&af)[QTM], const f16x8 (&bf)[TN], int mh) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < QTM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[mh * QTM + i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[j], af[i], acc[mh * QTM + i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  const int nk = g.K / BK;  // >= 2
  f16x8 fx[QTM], fy[QTM], fb0[TN], fb1[TN];
  auto ktile = [&](int kt, auto mode_tag) {
    constexpr int MODE = decltype(mode_tag)::value;
    const int h0 = 4 * kt;
    const f16* ia = slot(h0 + 2 + wm);
    const f16* ib = slot(h0 + (wn >> 1));
    read_a(fx, ia, 0, foff0);
    read_b(fb0, ib, foff0);
    if constexpr (MODE <= 1) issue(h0 + E, m0, n0);
    lds_barrier();
    mma(fx, fb0, 0);
    lds_barrier();
    read_a(fy, ia, 1, foff0);
    if constexpr (MODE <= 1) issue(h0 + E + 1, m0, n0);
    lds_barrier();
    mma(fy, fb0, 1);
    lds_barrier();
    read_a(fx, ia, 1, foff1);
    read_b(fb1, ib, foff1);
    if constexpr (MODE == 0) issue(h0 + E + 2, m0, n0);
    lds_barrier();
    mma(fx, fb1, 1);
    lds_barrier();
    read_a(fy, ia, 0, foff1);
    if constexpr (MODE == 0) {
      issue(h0 + E + 3, m0, n0);
      wait_vmcnt<2 * 2>();
    } else if constexpr (MODE == 1) {
      wait_vmcnt<0>();
    }
    lds_barrier();
    mma(fy, fb1, 0);
    lds_barrier();
  };

  tile_at(k, m0, n0);
#pragma unroll
  for (int h = 0; h < E; ++h) issue(h, m0, n0);
  wait_vmcnt<2 * 2>();
  lds_barrier();
  if (wm == 1) lds_barrier();  // the stagger
#pragma unroll 1
  for (;;) {
    f16x4 bv[TN];
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_RESID || EPI == EPI_BIAS_GELU)
        bv[j] = *(const f16x4*)(g.bias + n0 + wn * WTN + j * 16 + 4 * fg);
      else
        bv[j] = f16x4{};
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = (f32x4){0.f, 0.f, 0.f, 0.f};
    for (int kt = 0; kt < nk - 2; ++kt) ktile(kt, std::integral_constant<int, 0>{});
    ktile(nk - 2, std::integral_constant<int, 1>{});
    ktile(nk - 1, std::integral_constant<int, 2>{});
    if (wm == 0) lds_barrier();  // even out the barrier count: every wave is past its last ring read
    const int kn = k + nl;
    const bool more = kn < psize;
    int m1 = 0, n1 = 0;
    if (more) tile_at(kn, m1, n1);
    if (more) {  // the next tile's prologue, under this tile's epilogue
#pragma unroll
      for (int h = 0; h < E; ++h) issue(h, m1, n1);
    }
    epilogue_staged8p<EPI>(g, lds + 6 * HALF, acc, bv, m0, n0, wm, wn, tid, fr, fg, c_rsrc, x_rsrc);
    if (!more) break;
    // the next tile's first K-tile: all but its last two half-tiles' loads and this epilogue's stores
    if (EPI == EPI_BIAS_GELU && g.aux_out) wait_vmcnt<2 * 2 + 32>();
    else wait_vmcnt<2 * 2 + 16>();
    lds_barrier();
    if (wm == 1) lds_barrier();  // the stagger
    k = kn;
    m0 = m1;
    n0 = n1;
  }
}

int launch_tile8f(const GemmArgs& a, int epi, hipStream_t st);

int launch_tile8p(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + 255) / 256) * (a.N / 256);
  const int grid = std::min(tiles, mf_cu_count()) / 8 * 8;
  if (epi == EPI_F32 || !a.vec8 || a.N % 256 || grid < 8 || (int64_t)a.M * a.ldc * 2 >= (1ll << 31) ||
      (int64_t)a.M * a.ld_aux * 2 >= (1ll << 31))
    return mf_set_error("mf_gemm: persistent 256x256 tile needs fp16 C, N % 256 == 0, >= 8 tiles, < 2 GB", -2);
  switch (epi) {
    case EPI_NONE: gemm8p_kernel<EPI_NONE><<<grid, 512, 0, st>>>(a); break;
    case EPI_BIAS: gemm8p_kernel<EPI_BIAS><<<grid, 512, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm8p_kernel<EPI_BIAS_GELU><<<grid, 512, 0, st>>>(a); break;
    default: return launch_tile8f(a, epi, st);  // residual / QuickGELU' epilogues: gemm8f (bit-identical)
  }
  MF_CHECK_LAUNCH();
  return 0;
}

int launch_tile8s(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  dim3 grid(tiles), block(512);
  switch (epi) {
    case EPI_NONE: gemm8s_kernel<EPI_NONE><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: gemm8s_kernel<EPI_BIAS><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RESID: gemm8s_kernel<EPI_BIAS_RESID><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm8s_kernel<EPI_BIAS_GELU><<<grid, block, 0, st>>>(a); break;
    case EPI_DGELU: gemm8s_kernel<EPI_DGELU><<<grid, block, 0, st>>>(a); break;
    case EPI_F32: gemm8s_kernel<EPI_F32><<<grid, block, 0, st>>>(a); break;
    case EPI_RESID: gemm8s_kernel<EPI_RESID><<<grid, block, 0, st>>>(a); break;
    default: return mf_set_error("mf_gemm_nt: bad epilogue", -2);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

int launch_tile8f(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + 255) / 256) * ((a.N + 255) / 256);
  dim3 grid(tiles), block(512);
  switch (epi) {
    case EPI_NONE: gemm8f_kernel<EPI_NONE><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: gemm8f_kernel<EPI_BIAS><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RESID: gemm8f_kernel<EPI_BIAS_RESID><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm8f_kernel<EPI_BIAS_GELU><<<grid, block, 0, st>>>(a); break;
    case EPI_DGELU: gemm8f_kernel<EPI_DGELU><<<grid, block, 0, st>>>(a); break;
    case EPI_F32: gemm8f_kernel<EPI_F32><<<grid, block, 0, st>>>(a); break;
    case EPI_RESID: gemm8f_kernel<EPI_RESID><<<grid, block, 0, st>>>(a); break;
    default: return mf_set_error("mf_gemm_nt: bad epilogue", -2);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN>
int launch_tile8(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  dim3 grid(tiles), block(512);
  switch (epi) {
    case EPI_NONE: gemm8_kernel<BM, BN, WM, WN, EPI_NONE><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: gemm8_kernel<BM, BN, WM, WN, EPI_BIAS><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RESID: gemm8_kernel<BM, BN, WM, WN, EPI_BIAS_RESID><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm8_kernel<BM, BN, WM, WN, EPI_BIAS_GELU><<<grid, block, 0, st>>>(a); break;
    case EPI_DGELU: gemm8_kernel<BM, BN, WM, WN, EPI_DGELU><<<grid, block, 0, st>>>(a); break;
    case EPI_F32: gemm8_kernel<BM, BN, WM, WN, EPI_F32><<<grid, block, 0, st>>>(a); break;
    case EPI_RESID: gemm8_kernel<BM, BN, WM, WN, EPI_RESID><<<grid, block, 0, st>>>(a); break;
    default: return mf_set_error("mf_gemm_nt: bad epilogue", -2);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

template <int BM, int BN, int WM, int WN, int S, bool TA = false, bool TB = false>
int launch_tile(const GemmArgs& a, int epi, hipStream_t st) {
  const int tiles = ((a.M + BM - 1) / BM) * ((a.N + BN - 1) / BN);
  const int splits = a.ksplit > 0 ? (a.K + a.ksplit - 1) / a.ksplit : 1;
  dim3 grid(tiles * splits), block(WM * WN * 64);
  switch (epi) {
    case EPI_NONE: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_NONE, TA, TB><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_BIAS, TA, TB><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_RESID: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_BIAS_RESID, TA, TB><<<grid, block, 0, st>>>(a); break;
    case EPI_BIAS_GELU: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_BIAS_GELU, TA, TB><<<grid, block, 0, st>>>(a); break;
    case EPI_DGELU: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_DGELU, TA, TB><<<grid, block, 0, st>>>(a); break;
    case EPI_F32: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_F32, TA, TB><<<grid, block, 0, st>>>(a); break;
    case EPI_RESID: gemm_nt_kernel<BM, BN, WM, WN, S, EPI_RESID, TA, TB><<<grid, block, 0, st>>>(a); break;
    default: return mf_set_error("mf_gemm: bad epilogue", -2);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

// K-major operand combinations run on the 4-wave kernel's 128x128 / 128x64 / 64x64 tiles (a plain
// function: kernel templates instantiated only through nested function templates lose their host
// stubs under hipcc)
int launch_kmajor(const GemmArgs& a, bool ta, bool tb, int epi, int tile, hipStream_t st) {
#define MF_KM(TA_, TB_)                                                             \
  switch (tile) {                                                                   \
    case 1: return launch_tile<128, 128, 2, 2, 2, TA_, TB_>(a, epi, st);            \
    case 2: return launch_tile<128, 64, 2, 2, 2, TA_, TB_>(a, epi, st);             \
    case 3: return launch_tile<64, 64, 2, 2, 2, TA_, TB_>(a, epi, st);              \
    default: return mf_set_error("mf_gemm: K-major operands need tile 0-3", -2);    \
  }
  if (ta && tb) { MF_KM(true, true) }
  if (ta) { MF_KM(true, false) }
  MF_KM(false, true)
#undef MF_KM
}

// Tile -1 = "off the critical path": the products of the tower that runs beside the one setting the step
// (the engine passes it: the text tower at c4, the vision tower at C5).  That tower's own latency has slack
// (c4: text alone 2.46 ms against the vision tower's 4.80 ms, tests/diagnostics/tower_bound_probe.py), but its
// kernels' CU time is taken from the critical tower's kernels (the c4 step is 5.73 ms, not 4.80).  So its
// products want the tile that does the most work per CU-second, not the lowest latency: 160x128 for every
// row-major product of >= 2 048 rows (c4 text: 76..304 workgroups instead of the latency picks' 96x64 / 96x128
// and hipBLASLt's 64x96, 248..744 workgroups): c4 step +2.9 % (same-box A/B, two rounds: 5 585 / 5 617 ->
// 5 770 / 5 758 img/s; profiles/r03_v7_text_tile_ab.txt); C5 vision +0.6..0.8 %.
constexpr int kSideTile = 10;

// XCD blocking (tile_of): the N-range count 2^xb minimising one XCD's operand footprint A/(8/2^xb) +
// B/2^xb (bytes of the A rows and B rows it reads)
inline int gemm_xcd_split(int M, int N, int K) {
  const double a_bytes = 2.0 * M * K, b_bytes = 2.0 * N * K;
  int best = 0;
  double best_fp = 1e300;
  for (int xb = 0; xb <= 3; ++xb) {
    const double fp = a_bytes / (8 >> xb) + b_bytes / (1 << xb);
    if (fp < best_fp * 0.999) best = xb, best_fp = fp;
  }
  return best;
}

// automatic split count (tests/diagnostics/splitk_bench.py on the MaPLe dW shapes, K = 2926..6368):
// >= 144 128x128 tiles run best unsplit; 64..143 tiles on 4 slices; fewer on 8
// split count of a K-major weight gradient by its 128x128 output-tile count (tests/diagnostics/splitk_bench.py,
// r02: 144 tiles (block 11's c_fc / c_proj dW, K = 6368) 3 splits 52.7 us against 65 us single-pass)
inline int splitk_auto(int64_t tiles) { return tiles >= 256 ? 1 : (tiles >= 128 ? 3 : (tiles >= 64 ? 4 : 8)); }

// split-K combine: C[m][n] = sum_{s=0..S-1} ws[s][m][n] in that order (deterministic), fp16 or fp32 out.
// 4 columns per thread (N % 4 == 0).
__global__ void splitk_reduce_kernel(const float* __restrict__ ws, int S, int M, int N, void* __restrict__ C,
                                     int64_t ldc, int out_f16) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t nq = (int64_t)M * (N / 4);
  if (t >= nq) return;
  const int64_t m = t / (N / 4);
  const int n = (int)(t % (N / 4)) * 4;
  const int64_t plane = (int64_t)M * N;
  f32x4 acc = *(const f32x4*)(ws + m * N + n);
  for (int z = 1; z < S; ++z) {
    const f32x4 v = *(const f32x4*)(ws + z * plane + m * N + n);
    acc = (f32x4){acc[0] + v[0], acc[1] + v[1], acc[2] + v[2], acc[3] + v[3]};
  }
  if (out_f16) {
    f16x4 o = {(f16)acc[0], (f16)acc[1], (f16)acc[2], (f16)acc[3]};
    *(f16x4*)((f16*)C + m * ldc + n) = o;
  } else {
    *(f32x4*)((float*)C + m * ldc + n) = acc;
  }
}

}  // namespace

// C[M,N] = epilogue(op(A) . op(B)^T):  a_kmajor = 0: A[m][k] at A[m*lda + k], 1: A[k*lda + m];
// b_kmajor = 0: B[n][k] at B[n*ldb + k], 1: B[k*ldb + n].
extern "C" int mf_gemm(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb, int b_kmajor, void* C,
                       int64_t ldc, int M, int N, int K, const void* bias, const void* aux_in, void* aux_out,
                       int64_t ld_aux, int epilogue, int tile, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  const bool both_k = a_kmajor && b_kmajor;
  if (K <= 0 || (!both_k && (K % BK) != 0))
    return mf_set_error("mf_gemm: K must be a positive multiple of 64 unless both operands are K-major", -1);
  if ((N % 4) != 0 || (lda % 8) || (ldb % 8) || (ldc % 4)) return mf_set_error("mf_gemm: alignment", -1);
  if ((a_kmajor && (M % 8 || lda < M)) || (b_kmajor && (N % 8 || ldb < N)) || (!a_kmajor && lda < K) ||
      (!b_kmajor && ldb < K))
    return mf_set_error("mf_gemm: K-major operands need rows % 8 == 0 and ld >= rows; row-major ld >= K", -1);
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16) return mf_set_error("mf_gemm: operands must be 16-byte aligned", -1);
  if ((epilogue == EPI_BIAS || epilogue == EPI_BIAS_RESID || epilogue == EPI_BIAS_GELU) && !bias)
    return mf_set_error("mf_gemm: epilogue needs bias", -1);
  if ((epilogue == EPI_BIAS_RESID || epilogue == EPI_DGELU || epilogue == EPI_RESID) && !aux_in)
    return mf_set_error("mf_gemm: epilogue needs aux_in", -1);
  const int vec8 = (ldc % 8 == 0) && (ld_aux % 8 == 0) && ((uintptr_t)C % 16 == 0) &&
                   (!aux_in || (uintptr_t)aux_in % 16 == 0) && (!aux_out || (uintptr_t)aux_out % 16 == 0);
  GemmArgs a{(const f16*)A, (const f16*)B, C, (const f16*)bias, (const f16*)aux_in, (f16*)aux_out,
             lda, ldb, ldc, ld_aux, M, N, K, vec8, 0, gemm_xcd_split(M, N, K)};
  hipStream_t st = (hipStream_t)stream;
  const int64_t t128 = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (a_kmajor || b_kmajor) {
    if (tile <= 0) tile = t128 >= 512 ? 1 : (t128 >= 256 ? 2 : 3);
    return launch_kmajor(a, a_kmajor != 0, b_kmajor != 0, epilogue, tile, st);
  }
  // tile -1: a product of the tower off the step's critical path (throughput tiles, see text_tile)
  const bool side = tile == -1 && M >= 2048;
  if (tile == -1) tile = side ? kSideTile : 0;
  if (tile == 0) {  // heuristic: fill the 256 CUs (measured: tests/diagnostics/gemm_bench.py, gemm_stamps.cpp)
    const int64_t t256 = (int64_t)((M + 255) / 256) * ((N + 255) / 256);
    if (t256 >= 192 && t256 <= 256 && K >= 512)
      tile = 40;  // one round of 256x256 tiles on one workgroup per CU (vision QKV: 225 tiles), gemm8s
    else if (M >= 16384 && K >= 512)  // the C5 text tower (M = 77 000): many rounds of tiles whatever the
      // shape, so the tile's own efficiency decides (gemm_bench.py ... c5): the full-line 256x256 kernel for
      // N >= 1536 or K >= 1024 (r05, profiles/r05_v1_gemm8f_c5.txt: c5.dh 878 -> 946, c5.dqkv 832 -> 905, c5.proj
      // 827 -> 875, c5.fc 591 -> 612 TFLOP/s), 160x128 for the N = 512, K = 512 products (c5.out 623 / 581, c5.do
      // 735 / 663 on 160x128 / 256x256); r06: the eval engine's out-projection (M = 79 600 at EVAL_GROUP 4, N = K =
      // 768) 711..741 on 256x256 against 692..700 on 160x128 (profiles/r06_v1_gemm_eval4_*.txt, r06_v2_*)
      tile = (N >= 1536 || K >= 1024 || (N >= 768 && K >= 768)) ? 40 : 10;
      // r06: the persistent gemm8p (tile 41) is faster isolated on these launches (eval4 qkv 951 -> 975, fc 811 ->
      // 858, c5.qkv 789 -> 842 TFLOP/s, profiles/r06_v7_gemm8p_*.txt) but slower in the engine: eval pass 22 700 ->
      // 20 900 img/s, C5 1 261 -> 1 145 img/s (same box, interleaved, profiles/r06_v8_gemm8p_engine_ab.txt), so
      // it is not routed
    else if (M >= 4096 && K >= 512)  // vision products (M = 6368), tests/diagnostics/gemm_bench.py:
      // N = 3072: 160x128 (960 tiles); N = 768: 96x128 (402 tiles, two workgroups per CU) for K >= 2048,
      // 160x64 (480 tiles) for K = 768; +6..37 % over the 128-row tiles
      tile = N > 1024 ? 10 : (K >= 2048 ? 15 : 16);
    else if (M >= 2048 && N >= 1024 && K <= 768)
      tile = N >= 2048 ? 15 : 26;  // text (M = 2926): c_fc and its dX on 96x128, QKV on 96x64
    else if (M >= 2048 && N <= 768 && K >= 512)
      tile = 26;  // text N = 512 products (out-proj, c_proj, their dX, dQKV): 96x64, 248 tiles, +5..20 % over 64x64
    else if (M < 2048 && K >= 512) {
      // the small clients' products (C2 / C3: B = 4 images, 796 rows; K = 10 classes, 770 rows), r04 sweep
      // (gemm_bench.py ... c3, profiles/r04_v12_gemm_c3_tiles.txt): the long-K products run few tiles whose
      // K loops are latency-bound, so a 4-stage ring (64x64, or 32x64 when 64x64 gives < 128 tiles) is
      // +8..57 % (c_proj / c_fc dX / QKV dX); the wide ones take 96x64 (vision c_fc and its dX, text QKV)
      const int64_t t64 = (int64_t)((M + 63) / 64) * ((N + 63) / 64);
      if (K >= 1536) tile = t64 >= 128 ? 31 : 33;
      else if (N >= 3072 || (N > 1024 && N < 2048)) tile = 26;
      else tile = 3;
    } else
      tile = t128 >= 512 ? 1 : (t128 >= 256 ? 2 : 3);
  }
  // tile ids: the ones the heuristic picks (1, 2, 3, 10, 15, 16, 26, 31, 33, 40 = gemm8f, 41 = gemm8p), plus 11 (160x128 with a
  // 3-stage ring), 20 (gemm8s, the [256][32]-image 256x256 kernel gemm8f replaced in r05), 21 (8-wave 256x128) and
  // 22 (the unstaggered gemm8 at 256x256) as A/B baselines (tests/diagnostics/gemm_bench.py); the sweep also covered
  // 128x192, 192x128, 128x160, 160x160, 224x128, 96x192, 64x128, 160x192, 192x192, 256x128 on 4 waves and 128x256 /
  // 128x128 on 8 waves (slower on every MaPLe shape); r05 (profiles/r05_v2..v4_*): 224x96 / 224x128 / 208x96 4-wave
  // one-round tiles, 8-wave full-line 160x128 / 192x128 / 128x128 / 96x192 (gemm8g) and a persistent gemm8f whose next
  // tile's loads precede the current tile's buffer-store epilogue (gemm8fp) -- none faster where it would be picked
  // (gemm8g 192x128 within +0..2 % on the c4 K >= 2 304 products; gemm8fp +3..+11 % on some C5 products and -4..-60 %
  // on others), removed
  switch (tile) {
    case 1: return launch_tile<128, 128, 2, 2, 2>(a, epilogue, st);
    case 2: return launch_tile<128, 64, 2, 2, 2>(a, epilogue, st);
    case 3: return launch_tile<64, 64, 2, 2, 2>(a, epilogue, st);
    case 10: return launch_tile<160, 128, 2, 2, 2>(a, epilogue, st);
    case 11: return launch_tile<160, 128, 2, 2, 3>(a, epilogue, st);
    case 15: return launch_tile<96, 128, 2, 2, 2>(a, epilogue, st);
    case 16: return launch_tile<160, 64, 2, 2, 2>(a, epilogue, st);
    case 26: return launch_tile<96, 64, 2, 2, 2>(a, epilogue, st);
    case 31: return launch_tile<64, 64, 2, 2, 4>(a, epilogue, st);
    case 33: return launch_tile<32, 64, 2, 2, 4>(a, epilogue, st);
    case 20: return K < 128 ? launch_tile<128, 128, 2, 2, 2>(a, epilogue, st) : launch_tile8s(a, epilogue, st);
    case 21: return K < 128 ? launch_tile<128, 128, 2, 2, 2>(a, epilogue, st) : launch_tile8<256, 128, 2, 4>(a, epilogue, st);
    case 22: return K < 128 ? launch_tile<128, 128, 2, 2, 2>(a, epilogue, st) : launch_tile8<256, 256, 2, 4>(a, epilogue, st);
    case 40: return K < 128 ? launch_tile<128, 128, 2, 2, 2>(a, epilogue, st) : launch_tile8f(a, epilogue, st);
    case 41: return K < 128 ? launch_tile<128, 128, 2, 2, 2>(a, epilogue, st) : launch_tile8p(a, epilogue, st);
    default: return mf_set_error("mf_gemm: bad tile id", -2);
  }
}

extern "C" int mf_gemm_nt(const void* A, int64_t lda, const void* B, int64_t ldb, void* C, int64_t ldc, int M,
                          int N, int K, const void* bias, const void* aux_in, void* aux_out, int64_t ld_aux,
                          int epilogue, int tile, void* stream) {
  return mf_gemm(A, lda, 0, B, ldb, 0, C, ldc, M, N, K, bias, aux_in, aux_out, ld_aux, epilogue, tile, stream);
}

// Split-K plain product C = op(A) . op(B)^T for few output tiles and a long K (the weight gradients
// dW = dY^T X, K = tokens): `splits` workgroups per 128x128 tile each reduce a K slice into an fp32
// plane of ws (splits * M * N floats), then one pass sums the planes in a fixed order into C (fp16
// when out_f16, else fp32).  splits <= 0 picks enough slices for ~2 workgroups per CU.
extern "C" int mf_gemm_splitk(const void* A, int64_t lda, int a_kmajor, const void* B, int64_t ldb, int b_kmajor,
                              void* C, int64_t ldc, int M, int N, int K, float* ws, int64_t ws_floats, int splits,
                              int out_f16, void* stream) {
  if (M <= 0 || N <= 0) return 0;
  const bool both_k = a_kmajor && b_kmajor;
  if (K <= 0 || (!both_k && (K % BK) != 0))
    return mf_set_error("mf_gemm_splitk: K must be a positive multiple of 64 unless both operands are K-major", -1);
  if ((N % 8) != 0 || (lda % 8) || (ldb % 8) || (ldc % 4)) return mf_set_error("mf_gemm_splitk: alignment", -1);
  if ((a_kmajor && (M % 8 || lda < M)) || (b_kmajor && (N % 8 || ldb < N)) || (!a_kmajor && lda < K) ||
      (!b_kmajor && ldb < K))
    return mf_set_error("mf_gemm_splitk: K-major operands need rows % 8 == 0 and ld >= rows; row-major ld >= K", -1);
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)ws % 16 || (uintptr_t)C % 16)
    return mf_set_error("mf_gemm_splitk: pointers must be 16-byte aligned", -1);
  const int64_t tiles = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (splits <= 0) splits = splitk_auto(tiles);
  int ks = (int)((((int64_t)K + splits - 1) / splits + BK - 1) / BK * BK);
  if (ks < BK) ks = BK;
  splits = (K + ks - 1) / ks;
  if ((int64_t)splits * M * N > ws_floats) return mf_set_error("mf_gemm_splitk: workspace too small", -1);
  hipStream_t st = (hipStream_t)stream;
  // workgroup order: slice-major positions with each slice's run along the longer tile dimension
  // (split_tile_of) for >= 96 output tiles, else the r02 order (slice = dispatch id / tiles).  Same-box A/B
  // (tests/diagnostics/splitk_bench.py, profiles/r03_v1_splitk_order_ab.txt, two runs each): slice-major
  // v.dW_proj 52.1 -> 48.1 us, v.dW_qkv 40.2 -> 38.4, v.dW_fc 51.6 -> 50.1; but v.dW_out (36 tiles x 8)
  // 25.2 -> 26.9 and t.dW_fc (64 tiles x 4) 22.2 -> 24.1.
  const bool slice_major = tiles >= 96;
  GemmArgs a{(const f16*)A, (const f16*)B, ws, nullptr, nullptr, nullptr, lda, ldb, (int64_t)N, 0, M, N, K, 1, ks,
             slice_major ? ((N > M) ? 1 : 0) : 2};
  int rc;
  if (a_kmajor && b_kmajor) rc = launch_tile<128, 128, 2, 2, 2, true, true>(a, EPI_F32, st);
  else if (a_kmajor) rc = launch_tile<128, 128, 2, 2, 2, true, false>(a, EPI_F32, st);
  else if (b_kmajor) rc = launch_tile<128, 128, 2, 2, 2, false, true>(a, EPI_F32, st);
  else rc = launch_tile<128, 128, 2, 2, 2>(a, EPI_F32, st);
  if (rc) return rc;
  const int64_t nq = (int64_t)M * (N / 4);
  splitk_reduce_kernel<<<(unsigned)((nq + 255) / 256), 256, 0, st>>>(ws, splits, M, N, C, ldc, out_f16);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_gemm_splitk_ws_floats(int M, int N, int K, int splits) {
  const int64_t tiles = (int64_t)((M + 127) / 128) * ((N + 127) / 128);
  if (splits <= 0) splits = splitk_auto(tiles);
  int ks = (int)((((int64_t)K + splits - 1) / splits + BK - 1) / BK * BK);
  if (ks < BK) ks = BK;
  splits = (K + ks - 1) / ks;
  const int64_t n = (int64_t)splits * M * N;
  return n > 0x7fffffff ? -1 : (int)n;
}
