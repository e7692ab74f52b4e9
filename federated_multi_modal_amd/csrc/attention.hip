// Multi-head self-attention core of both CLIP towers: the SDPA that
// nn.MultiheadAttention(need_weights=False) runs inside ResidualAttentionBlock_MaPLe.attention
// (clip/model.py:303-305), with the text tower's additive causal mask (clip/model.py:679-685).
//
// Layout: qkv is the in-projection output [N*L, 3*D] (row n*L+l; q|k|v blocks of D = H*64
// columns, head h at columns h*64..h*64+63 of each block), out / dout are [N*L, D].
// head_dim = 64, L <= 512 (vision 199, text 77; 231..455 on caption-carrying batches) so a whole
// head's K and V fit in LDS: no online rescaling is needed.  Numerics follow torch's CPU flash kernel for fp16: scores in fp32,
// scale 1/8 applied in fp32, P = exp(s - rowmax) in fp32, row sum from the fp32 P, P rounded to
// fp16 for the PV product (fp32 accumulate), out = fp16(acc * (1/sum)).
//
// MFMA v_mfma_f32_16x16x32_f16 throughout, issued so that the reduction axis of each product
// lands where the next product needs it:
//   fwd:  S^T = K Q^T  -> each lane owns one query, 4 keys per 16-key tile (row max/sum by two
//         shuffles); O^T = V^T P^T takes P straight from the accumulators (keys permuted
//         consistently in both operands), V^T fragments by ds_read_b64_tr_b16 from the
//         row-major LDS image; each lane then holds 4 consecutive output columns (8-B stores).
//   bwd:  L <= 224: one fused workgroup per head (dK, dV, then dQ from dS^T kept in LDS);
//         longer: dK/dV kernel (Q and dO for the head in LDS) and dQ kernel (K and V in LDS), P
//         recomputed from the saved LSE.
// Forward kernel: attn_fwd4_kernel (scores in registers; 257..512 rows with one 8-wave workgroup per CU).
// LDS images are [rows][64] fp16 with the 16-byte chunk XOR swizzle chunk ^ (row & 7).
#include <algorithm>
#include <cstdlib>

#include "mf_common.h"

namespace {

MF_DEV int sw_off(int row, int col) {  // element offset in a swizzled [rows][64] fp16 image
  return row * 64 + ((((col >> 3) ^ (row & 7))) << 3) + (col & 7);
}

// 16 lanes of a group read rows r0..r0+3 x cols c0..c0+15; lane i gets column c0+i.
MF_DEV f16x4 tr_read(const f16* img, int r0, int c0, int lane) {
  const int ii = lane & 15;
  const int row = r0 + (ii >> 2);
  const int col = c0 + 4 * (ii & 3);
  const f16* p = img + sw_off(row, col);
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(f16x4, v);
}

MF_DEV f16x8 cat8(f16x4 a, f16x4 b) {
  return (f16x8){a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
}

MF_DEV f16x8 ld_frag(const f16* img, int row, int chunk) {
  return *(const f16x8*)(img + row * 64 + ((chunk ^ (row & 7)) << 3));
}

// Stage rows [0, LP) of one head (column offset col0 inside the qkv-like row) into a swizzled
// [LP][64] LDS image by global_load_lds (16 B per lane, no VGPR round trip; all of a block's
// loads are in flight together and retired by one wait).  The LDS side of an LDS-DMA is
// lane-linear (8 rows x 128 B per wave instruction), so the chunk XOR swizzle is applied to the
// per-lane SOURCE address.  Rows >= L re-read row L-1 (finite data; the kernels mask them).
typedef __attribute__((address_space(3))) void* lds_ptr_t;
template <int LP>
MF_DEV void stage_rows(f16* img, const f16* base, int64_t ld, int L, int col0) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int lrow = lane >> 3, lchunk = (lane & 7) ^ lrow;
  for (int i = w; i < LP / 8; i += nw) {
    int row = i * 8 + lrow;
    row = row < L ? row : L - 1;
    __builtin_amdgcn_global_load_lds((const void*)(base + (int64_t)row * ld + col0 + lchunk * 8),
                                     (lds_ptr_t)(img + i * 8 * 64), 16, 0, 0);
  }
}
MF_DEV void stage_wait() {
  __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8));  // vmcnt(0): this wave's LDS-DMA landed
  __syncthreads();                                              // ... and every other wave's
}

constexpr float kScale = 0.125f;  // 1/sqrt(64), SDPA default

// In-kernel timeline stamps for diagnostics (tests/diagnostics/attn_stamps.cpp defines
// MF_ATTN_STAMPS); compiled out of libmapfed.so.
#ifdef MF_ATTN_STAMPS
__device__ unsigned long long* g_astamps;
#define MF_ASTAMP(slot)                                                                   \
  do {                                                                                    \
    if (threadIdx.x == 0 && blockIdx.y == 0) g_astamps[(size_t)blockIdx.x * 8 + (slot)] = __builtin_amdgcn_s_memrealtime(); \
  } while (0)
// every workgroup of a 2-D grid (fwd4): slot 7 = the hardware id (XCC / CU) at the start
#define MF_ASTAMP2(slot)                                                                  \
  do {                                                                                    \
    if (threadIdx.x == 0) {                                                               \
      const size_t wg_ = (size_t)blockIdx.x * gridDim.y + blockIdx.y;                     \
      g_astamps[wg_ * 8 + (slot)] = __builtin_amdgcn_s_memrealtime();                     \
      if ((slot) == 0) g_astamps[wg_ * 8 + 7] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11)); \
    }                                                                                     \
  } while (0)
#else
#define MF_ASTAMP(slot) \
  do {                  \
  } while (0)
#define MF_ASTAMP2(slot) \
  do {                   \
  } while (0)
#endif

// ---------------------------------------------------------------------------------------------
// s_waitcnt vmcnt(n) for a wave-uniform runtime n (the immediate must be a constant)
MF_DEV void wait_vmcnt(int n) {
  switch (n) {
    case 0: __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8)); break;
    case 1: __builtin_amdgcn_s_waitcnt((1 & 15) | (7 << 4) | (15 << 8)); break;
    case 2: __builtin_amdgcn_s_waitcnt((2 & 15) | (7 << 4) | (15 << 8)); break;
    case 3: __builtin_amdgcn_s_waitcnt((3 & 15) | (7 << 4) | (15 << 8)); break;
    case 4: __builtin_amdgcn_s_waitcnt((4 & 15) | (7 << 4) | (15 << 8)); break;
    case 5: __builtin_amdgcn_s_waitcnt((5 & 15) | (7 << 4) | (15 << 8)); break;
    case 6: __builtin_amdgcn_s_waitcnt((6 & 15) | (7 << 4) | (15 << 8)); break;
    default: __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8)); break;
  }
}

// One 16-query tile of attn_fwd4_kernel once its Q fragments are in registers: scores, softmax, P.V.
// koff: [s2][hf] flattened (4), voff: [dt][hf] flattened (8).  V_WAIT: the V image may still be
// landing; it is waited for (vmcnt 0 + workgroup barrier) between the softmax and P.V, so every wave
// of the workgroup calls this, active or not.
template <int LKP, bool CAUSAL, bool V_WAIT>
MF_DEV void fwd4_tile(const f16* sK, const f16* sV, const int* koff, const int* voff, f16x8 qf0, f16x8 qf1,
                      bool active, int q0, int L, int lane, f16* __restrict__ out, int64_t ld_out,
                      float* __restrict__ lse, int ld_lse, int64_t row0, int h, int nh) {
  constexpr int NKT = LKP / 16;
  constexpr int NKS = (LKP + 31) / 32;
  constexpr bool HALF = (LKP % 32) != 0;  // the last 32-key chunk has only its first 16 keys staged
  const int fr = lane & 15, fg = lane >> 4;
  const int q = q0 + fr;
  const int kt_end = CAUSAL ? min(NKT, (q0 + 16 + 15) / 16) : NKT;
  const int ks_end = (kt_end + 1) / 2;
  f32x4 sc[NKS][2];
  float m = -INFINITY;
  if (active) {
    // all scores: S^T tiles (key rows, this lane's query column), chunk ks = keys 32ks .. 32ks+31
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      sc[ks][0] = sc[ks][1] = (f32x4){-INFINITY, -INFINITY, -INFINITY, -INFINITY};
      if (ks < ks_end) {
        const f16* kb = sK + ks * 32 * 64;
        f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = {0.f, 0.f, 0.f, 0.f};
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)(kb + koff[0]), qf0, a0, 0, 0, 0);
        a0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)(kb + koff[2]), qf1, a0, 0, 0, 0);
        sc[ks][0] = a0;
        if (!(HALF && ks == NKS - 1)) {  // keys 32ks+16.. exist (else they stay -inf: P = 0)
          a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)(kb + koff[1]), qf0, a1, 0, 0, 0);
          a1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(*(const f16x8*)(kb + koff[3]), qf1, a1, 0, 0, 0);
          sc[ks][1] = a1;
        }
      }
      // keep at most two chunks of K fragments in flight (the compiler would hoist every read and
      // exceed the 128-VGPR budget of 16 waves per CU)
      if (ks & 1) asm volatile("" ::: "memory");
    }
    // every launch stages LKP = L rounded up to 16 keys (mf_attention_fwd / _rows), so L > LKP - 16: without the
    // causal mask only the chunks reaching past LKP - 16 can hold keys >= L, and the others skip the key test at
    // compile time
#pragma unroll
    for (int ks = 0; ks < NKS; ++ks) {
      if (ks < ks_end && (CAUSAL || (32 * ks + 32 > LKP - 15 && 32 * ks + 32 > L))) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int key0 = 32 * ks + 4 * fg + i, key1 = key0 + 16;
          if (key0 >= L || (CAUSAL && key0 > q)) sc[ks][0][i] = -INFINITY;
          if (key1 >= L || (CAUSAL && key1 > q) || 2 * ks + 1 >= kt_end) sc[ks][1][i] = -INFINITY;
        }
      }
      m = fmaxf(m, fmaxf(fmaxf(sc[ks][0][0], sc[ks][0][1]), fmaxf(sc[ks][0][2], sc[ks][0][3])));
      m = fmaxf(m, fmaxf(fmaxf(sc[ks][1][0], sc[ks][1][1]), fmaxf(sc[ks][1][2], sc[ks][1][3])));
    }
    m = fmaxf(m, __shfl_xor(m, 16, 64));
    m = fmaxf(m, __shfl_xor(m, 32, 64));
  }
  if (V_WAIT) stage_wait();  // V landed (this wave's DMA, then every wave's)
  if (!active) return;
  constexpr float kLog2eScale = 0.125f * 1.4426950408889634f;
  const float mb = -m * kLog2eScale;
  float l = 0.f;
  f32x4 oacc[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) oacc[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int ks = 0; ks < NKS; ++ks) {
    if (ks < ks_end) {
      f16x8 pf;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float p0 = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[ks][0][i], kLog2eScale, mb));
        const float p1 = __builtin_amdgcn_exp2f(__builtin_fmaf(sc[ks][1][i], kLog2eScale, mb));
        l += p0 + p1;
        pf[i] = (f16)p0;
        pf[4 + i] = (f16)p1;
      }
      const f16* vb = sV + ks * 32 * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        s16x4 v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(vb + voff[2 * dt]));
        s16x4 v1 = {0, 0, 0, 0};  // unstaged keys of a half chunk: V = 0 against P = 0
        if (!(HALF && ks == NKS - 1))
          v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(vb + voff[2 * dt + 1]));
        oacc[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(cat8(__builtin_bit_cast(f16x4, v0), __builtin_bit_cast(f16x4, v1)),
                                                          pf, oacc[dt], 0, 0, 0);
      }
    }
  }
  l += __shfl_xor(l, 16, 64);
  l += __shfl_xor(l, 32, 64);
  if (q < L) {
    const float inv = 1.0f / l;
    f16* orow = out + (row0 + q) * ld_out + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (f16)(oacc[dt][i] * inv);
      *(f16x4*)(orow + 16 * dt + 4 * fg) = o;
    }
    if (fg == 0) lse[(int64_t)nh * ld_lse + q] = m * kScale + __logf(l);
  }
}

// Forward, single pass with register-resident scores (16 queries per wave): every score of the wave's
// queries (LKP keys x 16 queries = LKP/4 fp32 per lane) is computed ONCE by independent back-to-back MFMAs
// and kept in registers; row max, exp, row sum and the fp16 P pack then run from registers, and P . V
// follows (bit-identical to the two-pass form it replaced in r02, with a third fewer MFMAs and K reads).
// Staging overlaps the first tile: its Q fragments are loaded first, then K, then V (LDS-DMA); the
// scores start once Q and K have landed (vmcnt = this wave's V loads) and V is waited for only before
// P.V, so the V transfer runs under the score MFMAs and the softmax.
// MAXT = 512 for 257..512 rows: one workgroup per CU (K / V of the head take up to 128 KB of LDS), so
// two waves per SIMD and a 256-VGPR budget for the LKP/4 register-resident scores per lane.
template <int LKP, bool CAUSAL, int MAXT = 1024>
__global__ __launch_bounds__(MAXT) void attn_fwd4_kernel(const f16* __restrict__ qkv, int64_t ld_qkv,
                                                           f16* __restrict__ out, int64_t ld_out,
                                                           float* __restrict__ lse, int ld_lse, int L, int H,
                                                           int Lq) {
  // Lq <= L: only query rows 0 .. Lq-1 of each head are computed (their tiles; a tile's rows past Lq still are,
  // bit for bit as in a full launch: every query's arithmetic is independent of the other tiles)
  __shared__ __attribute__((aligned(16))) f16 sK[LKP * 64];
  __shared__ __attribute__((aligned(16))) f16 sV[LKP * 64];
  const int D = H * 64;
  // (head, query split) of this workgroup.  257..512 rows (MAXT = 512, one workgroup per CU) with the heads a
  // multiple of 8: the gridDim.y splits of a head take dispatch ids 8 apart (the hardware deals consecutive ids
  // round-robin to the 8 XCDs), so they run on one XCD at the same time and the second staging of the head's K / V
  // finds it in that XCD's L2 (r06, tests/diagnostics/attn_bench.py: 455 rows 50 -> 45 us; at c4's 199 rows the
  // same pairing is slower, 13.8 -> 14.4 us, profiles/r06_v17_attn_split_pairing.txt)
  int nh = blockIdx.x, split = blockIdx.y;
  if (MAXT == 512 && gridDim.y > 1 && (gridDim.x & 7) == 0) {
    const int id = blockIdx.x + blockIdx.y * gridDim.x, per = 8 * gridDim.y;
    nh = (id / per) * 8 + (id & 7);
    split = (id % per) >> 3;
  }
  const int n = nh / H, h = nh % H;
  const f16* base = qkv + (int64_t)n * L * ld_qkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fr = lane & 15, fg = lane >> 4, ii = lane & 15;
  const int qstep = gridDim.y * nw * 16;
  int q0 = (split * nw + w) * 16;
  const bool active = q0 < Lq;
  MF_ASTAMP2(0);
  f16x8 qf0, qf1;
  {
    const int q = q0 + fr;
    const f16* qrow = base + (int64_t)(q < L ? q : L - 1) * ld_qkv + h * 64 + 8 * fg;
    qf0 = *(const f16x8*)qrow;
    qf1 = *(const f16x8*)(qrow + 32);
  }
  stage_rows<LKP>(sK, base, ld_qkv, L, D + h * 64);
  stage_rows<LKP>(sV, base, ld_qkv, L, 2 * D + h * 64);
  const int nv = w < LKP / 8 ? (LKP / 8 - w + nw - 1) / nw : 0;  // this wave's V loads (issued last)

  int koff[4], voff[8];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int row = 16 * hf + fr;
      koff[2 * s2 + hf] = row * 64 + (((4 * s2 + fg) ^ (row & 7)) << 3);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) voff[2 * dt + hf] = sw_off(16 * hf + 4 * fg + (ii >> 2), 16 * dt + 4 * (ii & 3));
  }
  wait_vmcnt(nv);   // Q and this wave's K landed
  __syncthreads();  // ... and every wave's K
  MF_ASTAMP2(1);
  fwd4_tile<LKP, CAUSAL, true>(sK, sV, koff, voff, qf0, qf1, active, q0, L, lane, out, ld_out, lse, ld_lse,
                               (int64_t)n * L, h, nh);
  MF_ASTAMP2(2);
  for (q0 += qstep; q0 < Lq; q0 += qstep) {
    const int q = q0 + fr;
    const f16* qrow = base + (int64_t)(q < L ? q : L - 1) * ld_qkv + h * 64 + 8 * fg;
    qf0 = *(const f16x8*)qrow;
    qf1 = *(const f16x8*)(qrow + 32);
    fwd4_tile<LKP, CAUSAL, false>(sK, sV, koff, voff, qf0, qf1, true, q0, L, lane, out, ld_out, lse, ld_lse,
                                  (int64_t)n * L, h, nh);
  }
  MF_ASTAMP2(3);
}

// ---------------------------------------------------------------------------------------------
// Fused in-projection + attention forward: qkv_h = x_n W_h^T + b_h followed by SDPA on it
// (ResidualAttentionBlock_MaPLe.attention -> nn.MultiheadAttention, clip/model.py:303-305: the
// in-projection GEMM and the attention core of one block in one launch).
//
// One workgroup per (sequence n, head h).  Phase 1 is the head's slice of the in-projection GEMM:
// [MR rows of x_n] x [192 rows of W_in: this head's q | k | v rows]^T, K = D, with the arithmetic of
// the standalone GEMM (gemm.hip) -- v_mfma_f32_16x16x32_f16 with the weight fragment as the first
// operand, k-subs of 32 in ascending k, fp16(acc + bias) -- so the q/k/v values are bit-identical to
// mf_gemm_nt's.  Operands stream HBM -> LDS by LDS-DMA through a ring of NR k-sub slots ([rows][32]
// images, 16-byte chunk c of row r at c ^ ((-(r >> 2)) & 3)), NR - 1 slots in flight.  Waves form a
// (MR/32) x 2 grid of 32-row x 96-column sub-tiles.  Rows past the sequence read the next sequence's
// rows (or zeros past the buffer): finite values whose keys the attention masks and whose queries are
// not stored.  Phase 2 writes the fp16 q / k / v of the head into swizzled [MR][64] LDS images (the
// ring is dead by then), stores them to `qkv` (the backward reads them), and runs the attention of
// fwd4_tile on them: one 16-query tile per wave, bit-identical to attn_fwd4_kernel.
// What the fusion removes: the qkv round trip through HBM between the two launches (the attention's
// K / V staging burst), one launch boundary, and the GEMM's chip-wide epilogue store burst (here the
// stores of a head overlap other workgroups' GEMM phases).
MF_DEV void wait_vm_n(int n) {  // s_waitcnt vmcnt(n), n wave-uniform in 0..15
  switch (n) {
#define MF_VMC(k) case k: __builtin_amdgcn_s_waitcnt((k & 15) | (7 << 4) | (15 << 8)); break;
    MF_VMC(0) MF_VMC(1) MF_VMC(2) MF_VMC(3) MF_VMC(4) MF_VMC(5) MF_VMC(6) MF_VMC(7)
    MF_VMC(8) MF_VMC(9) MF_VMC(10) MF_VMC(11) MF_VMC(12) MF_VMC(13) MF_VMC(14) MF_VMC(15)
#undef MF_VMC
    default: __builtin_amdgcn_s_waitcnt((0 & 15) | (7 << 4) | (15 << 8)); break;
  }
}

MF_DEV void lds_bar() {  // s_barrier with LDS ordering and no vmcnt(0): LDS-DMA stays in flight across it
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Forward, persistent over heads: each workgroup (one 16-query tile per wave, ceil(L/16) waves) walks heads
// blockIdx.x, + gridDim.x, ... with K / V double-buffered in LDS -- the next head's LDS-DMA is issued before the
// current head's tiles run, so from the second head on the staging hides under the tiles instead of every
// workgroup life starting with it.  Per tile the arithmetic of attn_fwd4_kernel (fwd4_tile): bit-identical.
template <int LKP, bool CAUSAL>
__global__ __launch_bounds__(1024) void attn_fwdp_kernel(const f16* __restrict__ qkv, int64_t ld_qkv,
                                                         f16* __restrict__ out, int64_t ld_out,
                                                         float* __restrict__ lse, int ld_lse, int L, int H, int NH) {
  __shared__ __attribute__((aligned(16))) f16 sK[2][LKP * 64];
  __shared__ __attribute__((aligned(16))) f16 sV[2][LKP * 64];
  const int D = H * 64;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  const int fr = lane & 15, fg = lane >> 4, ii = lane & 15;
  const int q0 = w * 16;
  const bool active = q0 < L;
  int koff[4], voff[8];
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      const int row = 16 * hf + fr;
      koff[2 * s2 + hf] = row * 64 + (((4 * s2 + fg) ^ (row & 7)) << 3);
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) voff[2 * dt + hf] = sw_off(16 * hf + 4 * fg + (ii >> 2), 16 * dt + 4 * (ii & 3));
  }
  // this wave's LDS-DMA instructions per head (K and V, stage_rows' row-group split)
  const int nkv = 2 * (w < LKP / 8 ? (LKP / 8 - w + nw - 1) / nw : 0);
  int nh = blockIdx.x;
  if (nh >= NH) return;
  {
    const f16* base = qkv + (int64_t)(nh / H) * L * ld_qkv;
    stage_rows<LKP>(sK[0], base, ld_qkv, L, D + (nh % H) * 64);
    stage_rows<LKP>(sV[0], base, ld_qkv, L, 2 * D + (nh % H) * 64);
  }
  for (int it = 0; nh < NH; ++it, nh += gridDim.x) {
    const int b = it & 1;
    const int n = nh / H, h = nh % H;
    const f16* base = qkv + (int64_t)n * L * ld_qkv;
    f16x8 qf0, qf1;
    {
      const int q = q0 + fr;
      const f16* qrow = base + (int64_t)(q < L ? q : L - 1) * ld_qkv + h * 64 + 8 * fg;
      qf0 = *(const f16x8*)qrow;
      qf1 = *(const f16x8*)(qrow + 32);
    }
    const int nn = nh + gridDim.x;
    int pend = 0;
    if (nn < NH) {  // the next head into the other buffer (free: the barrier closing the previous iteration)
      const f16* nb = qkv + (int64_t)(nn / H) * L * ld_qkv;
      stage_rows<LKP>(sK[b ^ 1], nb, ld_qkv, L, D + (nn % H) * 64);
      stage_rows<LKP>(sV[b ^ 1], nb, ld_qkv, L, 2 * D + (nn % H) * 64);
      pend = nkv;
    }
    wait_vm_n(pend);  // this head's K / V (issued an iteration earlier) and the Q fragments have landed
    lds_bar();        // ... for every wave
    fwd4_tile<LKP, CAUSAL, false>(sK[b], sV[b], koff, voff, qf0, qf1, active, q0, L, lane, out, ld_out, lse, ld_lse,
                                  (int64_t)n * L, h, nh);
    lds_bar();  // every wave is done with buffer b before the next iteration stages into it
  }
}

// one k-sub of the fused kernel's LDS-DMA: this wave's instructions u (x rows or W rows) into `slot`.  The
// buffer descriptors are built here from (pointer, byte range): a kernel template whose body holds a
// descriptor-typed lambda capture or parameter loses its host stub under hipcc (see gemm.hip dma_stage).
template <int IPW_MAX, int NW, int NI>
MF_DEV void qkv_dma_issue(const f16* x, int x_bytes, const f16* w, int w_bytes, f16* slot, const int* voff,
                          const int* dst, const bool* isx, int kbytes, int wid) {
  const auto x_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)x, 0, x_bytes, 0x00020000);
  const auto w_rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)w, 0, w_bytes, 0x00020000);
#pragma unroll
  for (int u = 0; u < IPW_MAX; ++u) {
    if (wid + NW * u < NI) {
      if (isx[u])
        __builtin_amdgcn_raw_ptr_buffer_load_lds(x_rsrc, (lds_ptr_t)(slot + dst[u]), 16, voff[u] + kbytes, 0, 0, 0);
      else
        __builtin_amdgcn_raw_ptr_buffer_load_lds(w_rsrc, (lds_ptr_t)(slot + dst[u]), 16, voff[u] + kbytes, 0, 0, 0);
    }
  }
}

template <int LKP, int MR, int D, bool CAUSAL, int NR>
MF_DEV void qkv_attn_fwd_body(const f16* __restrict__ x, int64_t ld_x, int x_rows, const f16* __restrict__ w,
                              const f16* __restrict__ bias, f16* __restrict__ qkv, int64_t ld_qkv,
                              f16* __restrict__ out, int64_t ld_out, float* __restrict__ lse, int ld_lse, int L,
                              int H) {
  constexpr int WMG = MR / 32, NW = 2 * WMG, NT = 64 * NW;
  constexpr int HK = 32, KS = 64, NKT = D / KS;  // k-subs of 32; a K-step (ring slot) holds two
  constexpr int NA = MR / 16, NB = 192 / 16;     // LDS-DMA wave instructions (16 rows x 64 B) per k-sub
  constexpr int NI = NA + NB;
  constexpr int IPW_MAX = (NI + NW - 1) / NW;
  constexpr int HALF = (MR + 192) * HK;          // one k-sub's [A | B] images
  constexpr int SLOT = 2 * HALF;                 // fp16 elements per ring slot (one K-step)
  constexpr int IMG = MR * 64;                   // one [MR][64] q / k / v image
  constexpr int RING = NR * SLOT;
  constexpr int LDS_ELEMS = RING > 3 * IMG ? RING : 3 * IMG;
  constexpr int P = NR - 1;                      // K-steps in flight
  static_assert(LDS_ELEMS * 2 <= 160 * 1024, "LDS");
  static_assert(LKP <= MR && LKP % 16 == 0 && LKP / 16 <= NW, "one attention tile per wave");
  static_assert(2 * IPW_MAX * (P - 1) <= 15, "vmcnt range");
  __shared__ __attribute__((aligned(1024))) f16 lds[LDS_ELEMS];

  // XCD-aware bijective remap (blocks are dealt round-robin over the 8 XCDs): each XCD takes a contiguous
  // range of (sequence, head) pairs, so the 12 heads of a sequence share its x rows in one L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, qq = nwg >> 3, rr = nwg & 7;
  const int nh = (xcd < rr ? xcd * (qq + 1) : rr * (qq + 1) + (xcd - rr) * qq) + (bid >> 3);
  const int n = nh / H, h = nh % H;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mg = wid >> 1, ng = wid & 1;
  const int fr = lane & 15, fg = lane >> 4;

  // LDS-DMA plan: wave instruction t (t = wid + NW*u) fills 16 rows of the slot: t < NA -> x rows
  // 16t.., else W rows of part (t-NA)/4 (q, k, v), 16 rows each
  const int x_bytes = (int)(((int64_t)(x_rows - 1) * ld_x + D) * 2);
  const int w_bytes = (int)(((int64_t)3 * D - 1) * D + D) * 2;
  const int src_chunk = (lane & 3) ^ ((-(lane >> 4)) & 3);
  int dma_voff[IPW_MAX], dma_dst[IPW_MAX];
  bool dma_x[IPW_MAX];
  int ipw = 0;
#pragma unroll
  for (int u = 0; u < IPW_MAX; ++u) {
    const int t = wid + NW * u;
    dma_x[u] = t < NA;
    if (t < NA) {
      const int row = 16 * t + (lane >> 2);
      dma_voff[u] = (int)((((int64_t)n * L + row) * ld_x + src_chunk * 8) * 2);
      dma_dst[u] = 16 * t * HK;
    } else {
      const int tb = t - NA, part = tb >> 2;
      const int wrow = part * D + h * 64 + 16 * (tb & 3) + (lane >> 2);
      dma_voff[u] = (int)(((int64_t)wrow * D + src_chunk * 8) * 2);
      dma_dst[u] = (MR + 16 * tb) * HK;
    }
    ipw += t < NI ? 1 : 0;
  }
#define MF_QKV_ISSUE(kt)                                                                                     \
  do {                                                                                                       \
    f16* s_ = lds + ((kt) % NR) * SLOT;                                                                      \
    qkv_dma_issue<IPW_MAX, NW, NI>(x, x_bytes, w, w_bytes, s_, dma_voff, dma_dst, dma_x, (kt) * KS * 2, wid); \
    qkv_dma_issue<IPW_MAX, NW, NI>(x, x_bytes, w, w_bytes, s_ + HALF, dma_voff, dma_dst, dma_x,              \
                                   (kt) * KS * 2 + HK * 2, wid);                                             \
  } while (0)

  f32x4 acc[2][6];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) acc[i][jj] = (f32x4){0.f, 0.f, 0.f, 0.f};

  MF_ASTAMP2(0);
#pragma unroll
  for (int kt = 0; kt < P; ++kt) MF_QKV_ISSUE(kt);
  const int frag_off = fr * HK + ((fg ^ ((-(fr >> 2)) & 3)) << 3);
#pragma unroll 1
  for (int kt = 0; kt < NKT; ++kt) {
    // this wave's DMA of K-step kt landed (the younger in-flight K-steps may stay), then every wave's
    wait_vm_n(2 * ipw * min(P - 1, NKT - 1 - kt));
    lds_bar();
    if (kt + P < NKT) MF_QKV_ISSUE(kt + P);
#pragma unroll
    for (int s = 0; s < 2; ++s) {  // k-subs in ascending k (the standalone GEMM's accumulation order)
      const f16* sa = lds + (kt % NR) * SLOT + s * HALF;
      const f16* sb = sa + MR * HK;
      f16x8 af[2], bf[6];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *(const f16x8*)(sa + (32 * mg + 16 * i) * HK + frag_off);
#pragma unroll
      for (int jj = 0; jj < 6; ++jj) bf[jj] = *(const f16x8*)(sb + (16 * (6 * ng + jj)) * HK + frag_off);
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int jj = 0; jj < 6; ++jj)
          acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_f16(bf[jj], af[i], acc[i][jj], 0, 0, 0);
    }
  }
  MF_ASTAMP2(1);
  // bias of this lane's output columns, loaded after the K loop (12 VGPRs the loop does not hold: the text
  // kernel fits 128 VGPRs with it out of the loop); its latency overlaps the barrier
  f16x4 bv[6];
#pragma unroll
  for (int jj = 0; jj < 6; ++jj) {
    const int j = 6 * ng + jj;
    bv[jj] = *(const f16x4*)(bias + (j >> 2) * D + h * 64 + 16 * (j & 3) + 4 * fg);
  }
  __syncthreads();  // every wave is done with the ring

  // q / k / v images: fp16(acc + bias) (the GEMM's EPI_BIAS rounding); lane holds row
  // 32mg + 16i + fr, columns 16j + 4fg .. +3 of the head's 192
  f16* sQ = lds;
  f16* sK = lds + IMG;
  f16* sV = lds + 2 * IMG;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 32 * mg + 16 * i + fr;
#pragma unroll
    for (int jj = 0; jj < 6; ++jj) {
      const int j = 6 * ng + jj;
      f16x4 t;
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] = (f16)(acc[i][jj][e] + (float)bv[jj][e]);
      *(f16x4*)(lds + (j >> 2) * IMG + sw_off(r, 16 * (j & 3) + 4 * fg)) = t;
    }
  }
  __syncthreads();
  MF_ASTAMP2(2);
  // the head's q | k | v rows to HBM (the backward's operands), 16 B per access
  for (int t = tid; t < L * 24; t += NT) {
    const int r = t / 24, pc = t - 24 * r, part = pc >> 3, c = pc & 7;
    const f16x8 v = *(const f16x8*)(lds + part * IMG + sw_off(r, 8 * c));
    *(f16x8*)(qkv + ((int64_t)n * L + r) * ld_qkv + part * D + h * 64 + 8 * c) = v;
  }
  // attention: wave w takes queries 16w .. 16w+15
  if (wid < LKP / 16) {
    const int q0 = 16 * wid, ii = lane & 15;
    int koff[4], voff[8];
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const int row = 16 * hf + fr;
        koff[2 * s2 + hf] = row * 64 + (((4 * s2 + fg) ^ (row & 7)) << 3);
      }
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) voff[2 * dt + hf] = sw_off(16 * hf + 4 * fg + (ii >> 2), 16 * dt + 4 * (ii & 3));
    }
    const f16x8 qf0 = ld_frag(sQ, q0 + fr, fg), qf1 = ld_frag(sQ, q0 + fr, 4 + fg);
    fwd4_tile<LKP, CAUSAL, false>(sK, sV, koff, voff, qf0, qf1, true, q0, L, lane, out, ld_out, lse, ld_lse,
                                  (int64_t)n * L, h, nh);
  }
  MF_ASTAMP2(3);
}

#define MF_QKV_ARGS                                                                                              \
  const f16 *__restrict__ x, int64_t ld_x, int x_rows, const f16 *__restrict__ w, const f16 *__restrict__ bias, \
      f16 *__restrict__ qkv, int64_t ld_qkv, f16 *__restrict__ out, int64_t ld_out, float *__restrict__ lse,    \
      int ld_lse, int L, int H
// vision (D = 768, 193..208 rows): 14 waves, the 160 KB ring: one workgroup per CU
__global__ __launch_bounds__(896) void qkv_attn_fwd_vision_kernel(MF_QKV_ARGS) {
  qkv_attn_fwd_body<208, 224, 768, false, 3>(x, ld_x, x_rows, w, bias, qkv, ld_qkv, out, ld_out, lse, ld_lse, L, H);
}
// text (D = 512, causal, 65..80 rows): 6 waves and 72 KB of LDS, so two workgroups per CU by LDS -- but only
// if no SIMD needs a 4th wave: waves are dealt to the SIMDs cyclically from a varying start, so the second
// workgroup's two-wave SIMDs can be the first's.  At 129 VGPRs (3 waves per SIMD) the stamps
// (tests/diagnostics/qkv_stamps.cpp) showed one workgroup per CU; at <= 128 (4 per SIMD: the bias load out
// of the K loop, 117 VGPRs) any placement fits.
__global__ __launch_bounds__(384) void qkv_attn_fwd_text_kernel(MF_QKV_ARGS) {
  qkv_attn_fwd_body<80, 96, 512, true, 2>(x, ld_x, x_rows, w, bias, qkv, ld_qkv, out, ld_out, lse, ld_lse, L, H);
}
#undef MF_QKV_ARGS

// Dq[nh][q] = sum_d dO[q][d] * O[q][d] (fp32) ------------------------------------------------
__global__ void attn_bwd_dot_kernel(const f16* __restrict__ out, int64_t ld_out, const f16* __restrict__ dout,
                                    int64_t ld_dout, float* __restrict__ dq_dot, int ld_lse, int N, int L, int H) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over N*H*L
  if (t >= (int64_t)N * H * L) return;
  const int q = t % L;
  const int nh = t / L;
  const int n = nh / H, h = nh % H;
  const f16* o = out + ((int64_t)n * L + q) * ld_out + h * 64;
  const f16* d = dout + ((int64_t)n * L + q) * ld_dout + h * 64;
  float s = 0.f;
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    f16x8 a = *(const f16x8*)(o + 8 * c), b = *(const f16x8*)(d + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) s += (float)a[e] * (float)b[e];
  }
  dq_dot[(int64_t)nh * ld_lse + q] = s;
}

// dK, dV: one workgroup per (n, h, 64-key block); each wave 16 keys, loops over all queries ----
template <int LQP, bool CAUSAL>
__global__ __launch_bounds__(512, 4) void attn_bwd_dkv_kernel(const f16* __restrict__ qkv, int64_t ld_qkv,
                                                          const f16* __restrict__ dout, int64_t ld_dout,
                                                          const float* __restrict__ lse,
                                                          const float* __restrict__ dq_dot, int ld_lse,
                                                          f16* __restrict__ dqkv, int64_t ld_dqkv, int L, int H) {
  __shared__ __attribute__((aligned(16))) f16 sQ[LQP * 64];
  __shared__ __attribute__((aligned(16))) f16 sdO[LQP * 64];
  __shared__ __attribute__((aligned(16))) float sL[LQP];
  __shared__ __attribute__((aligned(16))) float sD[LQP];
  const int D = H * 64;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const f16* base = qkv + (int64_t)n * L * ld_qkv;
  stage_rows<LQP>(sQ, base, ld_qkv, L, h * 64);
  stage_rows<LQP>(sdO, dout + (int64_t)n * L * ld_dout, ld_dout, L, h * 64);
  for (int i = threadIdx.x; i < LQP; i += blockDim.x) {
    sL[i] = i < L ? lse[(int64_t)nh * ld_lse + i] * 1.4426950408889634f : INFINITY;  // base 2; +inf masks
    sD[i] = i < L ? dq_dot[(int64_t)nh * ld_lse + i] : 0.f;
  }
  stage_wait();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // every wave takes 16-row tiles w, w + nw, ... of this head (the staged operands are shared)
  for (int k0 = (blockIdx.y * nw + w) * 16; k0 < L; k0 += gridDim.y * nw * 16) {
  const int fr = lane & 15, fg = lane >> 4;
  const int key = k0 + fr;
  const int kc = key < L ? key : L - 1;
  f16x8 kf[2], vf[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    kf[s] = *(const f16x8*)(base + (int64_t)kc * ld_qkv + D + h * 64 + 32 * s + 8 * fg);
    vf[s] = *(const f16x8*)(base + (int64_t)kc * ld_qkv + 2 * D + h * 64 + 32 * s + 8 * fg);
  }
  f32x4 dv[4], dk[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dv[dt] = dk[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};

#pragma unroll 1
  for (int qp = 0; qp < LQP / 32; ++qp) {
    if (CAUSAL && 32 * qp + 31 < k0) continue;  // every query < every key of this wave
    f16x8 pf, dsf;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int qt = 2 * qp + a;
      f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 qfr = ld_frag(sQ, qt * 16 + fr, 4 * s + fg);
        f16x8 ofr = ld_frag(sdO, qt * 16 + fr, 4 * s + fg);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(qfr, kf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ofr, vf[s], pacc, 0, 0, 0);
      }
      // the lane's 4 queries are consecutive: one 16-byte LDS read each for LSE and D
      const f32x4 l4 = *(const f32x4*)(sL + qt * 16 + 4 * fg);
      const f32x4 d4 = *(const f32x4*)(sD + qt * 16 + 4 * fg);
      constexpr float kScaleLog2e = 0.125f * 1.4426950408889634f;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int qq = qt * 16 + 4 * fg + i;
        const bool valid = key < L && !(CAUSAL && key > qq);  // qq >= L: LSE = +inf -> p = 0
        const float p = valid ? __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], kScaleLog2e, -l4[i])) : 0.f;
        const float ds = p * (pacc[i] - d4[i]);
        pf[a * 4 + i] = (f16)p;
        dsf[a * 4 + i] = (f16)ds;
      }
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f16x8 ao = cat8(tr_read(sdO, 32 * qp + 4 * fg, 16 * dt, lane), tr_read(sdO, 32 * qp + 16 + 4 * fg, 16 * dt, lane));
      dv[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ao, pf, dv[dt], 0, 0, 0);
      f16x8 aq = cat8(tr_read(sQ, 32 * qp + 4 * fg, 16 * dt, lane), tr_read(sQ, 32 * qp + 16 + 4 * fg, 16 * dt, lane));
      dk[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aq, dsf, dk[dt], 0, 0, 0);
    }
  }
  if (key < L) {
    f16* row = dqkv + ((int64_t)n * L + key) * ld_dqkv + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f16x4 ok, ov;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        ok[i] = (f16)(dk[dt][i] * kScale);
        ov[i] = (f16)dv[dt][i];
      }
      *(f16x4*)(row + D + 16 * dt + 4 * fg) = ok;
      *(f16x4*)(row + 2 * D + 16 * dt + 4 * fg) = ov;
    }
  }
  }
}

// dQ: one workgroup per (n, h, 64-query block); each wave 16 queries, loops over all keys -------
template <int LKP, bool CAUSAL>
__global__ __launch_bounds__(512, 4) void attn_bwd_dq_kernel(const f16* __restrict__ qkv, int64_t ld_qkv,
                                                         const f16* __restrict__ dout, int64_t ld_dout,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ dq_dot, int ld_lse,
                                                         f16* __restrict__ dqkv, int64_t ld_dqkv, int L, int H) {
  constexpr int NKT = LKP / 16;
  __shared__ __attribute__((aligned(16))) f16 sK[LKP * 64];
  __shared__ __attribute__((aligned(16))) f16 sV[LKP * 64];
  const int D = H * 64;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const f16* base = qkv + (int64_t)n * L * ld_qkv;
  stage_rows<LKP>(sK, base, ld_qkv, L, D + h * 64);
  stage_rows<LKP>(sV, base, ld_qkv, L, 2 * D + h * 64);
  stage_wait();

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, nw = blockDim.x >> 6;
  // every wave takes 16-row tiles w, w + nw, ... of this head (the staged operands are shared)
  for (int q0 = (blockIdx.y * nw + w) * 16; q0 < L; q0 += gridDim.y * nw * 16) {
  const int fr = lane & 15, fg = lane >> 4;
  const int q = q0 + fr;
  const int qc = q < L ? q : L - 1;
  f16x8 qf[2], of[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    qf[s] = *(const f16x8*)(base + (int64_t)qc * ld_qkv + h * 64 + 32 * s + 8 * fg);
    of[s] = *(const f16x8*)(dout + ((int64_t)n * L + qc) * ld_dout + h * 64 + 32 * s + 8 * fg);
  }
  const float lq = lse[(int64_t)nh * ld_lse + qc] * 1.4426950408889634f;  // base 2
  const float dq_d = dq_dot[(int64_t)nh * ld_lse + qc];
  f32x4 dq[4];
#pragma unroll
  for (int dt = 0; dt < 4; ++dt) dq[dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ks = 0; ks < NKT / 2; ++ks) {
    if (CAUSAL && 32 * ks > q0 + 15) break;
    f16x8 dsf;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int kt = 2 * ks + a;
      f32x4 sacc = {0.f, 0.f, 0.f, 0.f}, pacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        f16x8 kfr = ld_frag(sK, kt * 16 + fr, 4 * s + fg);
        f16x8 vfr = ld_frag(sV, kt * 16 + fr, 4 * s + fg);
        sacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(kfr, qf[s], sacc, 0, 0, 0);
        pacc = __builtin_amdgcn_mfma_f32_16x16x32_f16(vfr, of[s], pacc, 0, 0, 0);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int key = kt * 16 + 4 * fg + i;
        const bool valid = key < L && q < L && !(CAUSAL && key > q);
        const float p = valid ? __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[i], 0.125f * 1.4426950408889634f, -lq)) : 0.f;
        dsf[a * 4 + i] = (f16)(p * (pacc[i] - dq_d));
      }
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f16x8 ak = cat8(tr_read(sK, 32 * ks + 4 * fg, 16 * dt, lane), tr_read(sK, 32 * ks + 16 + 4 * fg, 16 * dt, lane));
      dq[dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ak, dsf, dq[dt], 0, 0, 0);
    }
  }
  if (q < L) {
    f16* row = dqkv + ((int64_t)n * L + q) * ld_dqkv + h * 64;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      f16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (f16)(dq[dt][i] * kScale);
      *(f16x4*)(row + 16 * dt + 4 * fg) = o;
    }
  }
  }
}

// Fused backward, one workgroup per (sequence, head), LP/32 waves, everything for the head in LDS:
//   phase 0: stage Q and dO (LDS-DMA), D[q] = sum_d dO[q][d] O[q][d] and LSE into LDS;
//   phase 1: wave w owns keys 32w..32w+31 (K, V fragments in registers) and sweeps the queries:
//            S^T-ordered P = exp(S*scale - LSE), dS = P (dP - D); dV += P^T dO, dK += dS^T Q, and
//            dS^T (fp16, the operand precision the dQ product uses) is written to LDS [key][q];
//   phase 2: K replaces Q in LDS, written from the waves' K fragments (no second fetch of K); wave w
//            owns queries 32w..32w+31: dQ = dS K from the stored dS^T (no recompute of S and dP, no
//            separate D kernel).
// LDS at LP = 224: Q 28 KB + dO 28 KB + dS^T 224 x 232 fp16 (101.5 KB) + LSE/D 1.75 KB = 159.25 KB.
template <int LP>
struct BwdLds {
  static constexpr int P = LP + 8;  // dS^T row pitch (elements)
  static constexpr int ELEMS = 2 * LP * 64 + LP * P + 2 * LP * 2;  // fp16 units (LSE, D as 2 fp16 each)
};

// 16 lanes of a group read rows r0..r0+3 x cols c0..c0+15 of a plain [rows][pitch] fp16 image;
// lane i of the group gets column c0+i (rows r0..r0+3 in its 4 elements)
MF_DEV f16x4 tr_read_p(const f16* img, int pitch, int r0, int c0, int lane) {
  const int ii = lane & 15;
  const f16* p = img + (r0 + (ii >> 2)) * pitch + c0 + 4 * (ii & 3);
  s16x4 v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p));
  return __builtin_bit_cast(f16x4, v);
}

template <int LP, bool CAUSAL, int KT>
__global__ __launch_bounds__(64 * (LP / (16 * KT))) void attn_bwd_fused_kernel(
    const f16* __restrict__ qkv, int64_t ld_qkv, const f16* __restrict__ out, int64_t ld_out,
    const f16* __restrict__ dout, int64_t ld_dout, const float* __restrict__ lse, int ld_lse,
    f16* __restrict__ dqkv, int64_t ld_dqkv, int L, int H) {
  constexpr int PT = BwdLds<LP>::P;
  __shared__ __attribute__((aligned(16))) f16 smem[BwdLds<LP>::ELEMS];
  f16* sQ = smem;                     // [LP][64] swizzled (phase 2: K)
  f16* sdO = smem + LP * 64;          // [LP][64] swizzled
  f16* sdST = smem + 2 * LP * 64;     // [LP keys][PT] plain
  float* sL = (float*)(sdST + LP * PT);
  float* sD = sL + LP;

  const int D = H * 64;
  const int nh = blockIdx.x, n = nh / H, h = nh % H;
  const f16* base = qkv + (int64_t)n * L * ld_qkv;
  const f16* obase = out + (int64_t)n * L * ld_out;
  const f16* dobase = dout + (int64_t)n * L * ld_dout;
  MF_ASTAMP(0);
  stage_rows<LP>(sQ, base, ld_qkv, L, h * 64);
  stage_rows<LP>(sdO, dobase, ld_dout, L, h * 64);

  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int fr = lane & 15, fg = lane >> 4;
  // phase 0: D and LSE of queries 16*KT*w .. +16*KT-1 (LPQ lanes per query, 64/LPQ dims each), from
  // global O and dO while the staging is in flight (reading dO back from LDS instead serialises D behind
  // the staging: +0.4 us per workgroup, tests/diagnostics/attn_stamps.cpp)
  {
    constexpr int LPQ = 4 / KT, DPL = 64 / LPQ;
    const int q = 16 * KT * w + lane / LPQ;
    const int part = lane % LPQ;
    float d = 0.f;
    if (q < L) {
      const f16* o = obase + (int64_t)q * ld_out + h * 64 + DPL * part;
      const f16* g = dobase + (int64_t)q * ld_dout + h * 64 + DPL * part;
#pragma unroll
      for (int c = 0; c < DPL / 8; ++c) {
        f16x8 a = *(const f16x8*)(o + 8 * c), b = *(const f16x8*)(g + 8 * c);
#pragma unroll
        for (int e = 0; e < 8; ++e) d += (float)a[e] * (float)b[e];
      }
    }
#pragma unroll
    for (int o2 = 1; o2 < LPQ; o2 <<= 1) d += __shfl_xor(d, o2, 64);
    if (part == 0) {
      sD[q] = q < L ? d : 0.f;
      // LSE in base 2 (P = exp2(S * scale * log2e - LSE * log2e)); +inf masks padded queries
      sL[q] = q < L ? lse[(int64_t)nh * ld_lse + q] * 1.4426950408889634f : INFINITY;
    }
  }
  // the wave's keys: K and V fragments straight to registers
  const int k0 = 16 * KT * w;
  f16x8 kf[KT][2], vf[KT][2];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int key = k0 + 16 * kt + fr;
    const int kc = key < L ? key : L - 1;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      kf[kt][s2] = *(const f16x8*)(base + (int64_t)kc * ld_qkv + D + h * 64 + 32 * s2 + 8 * fg);
      vf[kt][s2] = *(const f16x8*)(base + (int64_t)kc * ld_qkv + 2 * D + h * 64 + 32 * s2 + 8 * fg);
    }
  }
  stage_wait();  // Q, dO landed; D, LSE visible
  MF_ASTAMP(1);

  // ---- phase 1: dK, dV for keys k0..k0+31; dS^T -> LDS
  f32x4 dv[KT][4], dk[KT][4];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dv[kt][dt] = dk[kt][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int qp = 0; qp < LP / 32; ++qp) {
    if (CAUSAL && 32 * qp + 31 < k0) continue;  // (KT = 1 waves: k0 may sit mid-block)  // every query of the block precedes every key of the wave
    f16x8 pf[KT], dsf[KT];
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int qt = 2 * qp + a;
      f32x4 sacc[KT], pacc[KT];
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) sacc[kt] = pacc[kt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s2 = 0; s2 < 2; ++s2) {
        const f16x8 qfr = ld_frag(sQ, qt * 16 + fr, 4 * s2 + fg);
        const f16x8 ofr = ld_frag(sdO, qt * 16 + fr, 4 * s2 + fg);
#pragma unroll
        for (int kt = 0; kt < KT; ++kt) {
          sacc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(qfr, kf[kt][s2], sacc[kt], 0, 0, 0);
          pacc[kt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ofr, vf[kt][s2], pacc[kt], 0, 0, 0);
        }
      }
      // the lane's 4 queries are consecutive: one 16-byte LDS read each for LSE and D
      const f32x4 l4 = *(const f32x4*)(sL + qt * 16 + 4 * fg);
      const f32x4 d4 = *(const f32x4*)(sD + qt * 16 + 4 * fg);
      constexpr float kScaleLog2e = 0.125f * 1.4426950408889634f;
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        const int key = k0 + 16 * kt + fr;
        f16x4 dst;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int qq = qt * 16 + 4 * fg + i;
          const bool valid = key < L && !(CAUSAL && key > qq);  // qq >= L: LSE = +inf -> p = 0
          const float p = valid ? __builtin_amdgcn_exp2f(__builtin_fmaf(sacc[kt][i], kScaleLog2e, -l4[i])) : 0.f;
          const float ds = p * (pacc[kt][i] - d4[i]);
          pf[kt][a * 4 + i] = (f16)p;
          dsf[kt][a * 4 + i] = (f16)ds;
          dst[i] = (f16)ds;
        }
        *(f16x4*)(sdST + (k0 + 16 * kt + fr) * PT + qt * 16 + 4 * fg) = dst;
      }
    }
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f16x8 ao = cat8(tr_read(sdO, 32 * qp + 4 * fg, 16 * dt, lane), tr_read(sdO, 32 * qp + 16 + 4 * fg, 16 * dt, lane));
      const f16x8 aq = cat8(tr_read(sQ, 32 * qp + 4 * fg, 16 * dt, lane), tr_read(sQ, 32 * qp + 16 + 4 * fg, 16 * dt, lane));
#pragma unroll
      for (int kt = 0; kt < KT; ++kt) {
        dv[kt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ao, pf[kt], dv[kt][dt], 0, 0, 0);
        dk[kt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(aq, dsf[kt], dk[kt][dt], 0, 0, 0);
      }
    }
  }
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int key = k0 + 16 * kt + fr;
    if (key < L) {
      f16* row = dqkv + ((int64_t)n * L + key) * ld_dqkv + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        f16x4 ok, ov;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          ok[i] = (f16)(dk[kt][dt][i] * kScale);
          ov[i] = (f16)dv[kt][dt][i];
        }
        *(f16x4*)(row + D + 16 * dt + 4 * fg) = ok;
        *(f16x4*)(row + 2 * D + 16 * dt + 4 * fg) = ov;
      }
    }
  }

  MF_ASTAMP(2);
  // ---- phase 2: K into the Q region; dQ for queries q0..q0+16*KT-1 from dS^T
  __syncthreads();  // dS^T complete, every wave done reading Q / dO
  // the K image from the waves' own K fragments (rows k0.., the stage_rows layout: rows >= L hold row
  // L - 1), instead of fetching K again
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const int row = k0 + 16 * kt + fr;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) *(f16x8*)(sQ + row * 64 + (((4 * s2 + fg) ^ (row & 7)) << 3)) = kf[kt][s2];
  }
  __syncthreads();
  MF_ASTAMP(3);
  const f16* sK = sQ;
  const int q0 = 16 * KT * w;
  f32x4 dq[KT][4];
#pragma unroll
  for (int qt = 0; qt < KT; ++qt)
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) dq[qt][dt] = (f32x4){0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
  for (int ks = 0; ks < LP / 32; ++ks) {
    if (CAUSAL && 32 * ks > q0 + 16 * KT - 1) break;
    f16x8 dsf[KT];
#pragma unroll
    for (int qt = 0; qt < KT; ++qt)
      dsf[qt] = cat8(tr_read_p(sdST, PT, 32 * ks + 4 * fg, q0 + 16 * qt, lane),
                     tr_read_p(sdST, PT, 32 * ks + 16 + 4 * fg, q0 + 16 * qt, lane));
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) {
      const f16x8 ak = cat8(tr_read(sK, 32 * ks + 4 * fg, 16 * dt, lane), tr_read(sK, 32 * ks + 16 + 4 * fg, 16 * dt, lane));
#pragma unroll
      for (int qt = 0; qt < KT; ++qt) dq[qt][dt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(ak, dsf[qt], dq[qt][dt], 0, 0, 0);
    }
  }
#pragma unroll
  for (int qt = 0; qt < KT; ++qt) {
    const int q = q0 + 16 * qt + fr;
    if (q < L) {
      f16* row = dqkv + ((int64_t)n * L + q) * ld_dqkv + h * 64;
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        f16x4 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (f16)(dq[qt][dt][i] * kScale);
        *(f16x4*)(row + 16 * dt + 4 * fg) = o;
      }
    }
  }
  MF_ASTAMP(4);
}

#define MF_ATTN_DISPATCH(LP, CALL)                         \
  switch (LP) {                                            \
    case 32: CALL(32); break;                              \
    case 64: CALL(64); break;                              \
    case 96: CALL(96); break;                              \
    case 128: CALL(128); break;                            \
    case 160: CALL(160); break;                            \
    case 192: CALL(192); break;                            \
    case 224: CALL(224); break;                            \
    case 256: CALL(256); break;                            \
    default: return mf_set_error("attention: bad padded length", -1); \
  }

// Sequences of 257..512 rows (the vision tower under the caption path, 199 + 8*B rows at B = 32, J = 9):
// non-causal only, on the two-pass forward and the dK/dV + dQ backward with K / V (or Q / dO) of the head
// in LDS (128 KB at 512 rows, one workgroup per CU).
#define MF_ATTN_DISPATCH_LONG(LP, CALL)                           \
  switch (LP) {                                                   \
    case 288: CALL(288); break;                                   \
    case 320: CALL(320); break;                                   \
    case 352: CALL(352); break;                                   \
    case 384: CALL(384); break;                                   \
    case 416: CALL(416); break;                                   \
    case 448: CALL(448); break;                                   \
    case 480: CALL(480); break;                                   \
    case 512: CALL(512); break;                                   \
    default: return mf_set_error("attention: bad padded length", -1); \
  }

inline int padded_len(int L) { return ((L + 31) / 32) * 32; }
// one workgroup per (sequence, head): up to 8 waves sharing the staged operands, one 16-row tile each
inline int attn_threads(int L) { return 64 * std::max(1, std::min(8, (L + 15) / 16)); }
// query-tile split of a head over workgroups: enough workgroups to cover the chip (measured best:
// 2 at N*H = 384, 4 at N*H = 48; tests/diagnostics/attn_bench.py), at the cost of re-staging K/V.  Sequences
// longer than 128 rows keep at least 2 whatever the head count (r05: the eval engine's 4 800 heads): a whole
// 199-row head is a 13-wave workgroup, of which only one fits a CU (16 waves at 104 VGPRs), so its K/V staging
// never overlaps another workgroup's tiles; two 7-wave halves do fit, two per CU.
inline int attn_qsplit(int NH, int L) {
  const int want = std::max(L > 128 ? 2 : 1, std::min(4, (768 + NH - 1) / NH));
  return std::max(1, std::min(want, (L + 15) / 16 / 2));
}

}  // namespace

extern "C" int mf_attention_fwd(const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse, int ld_lse,
                                int N, int L, int H, int causal, void* stream) {
  if (N <= 0) return 0;
  if (L <= 0 || L > 512) return mf_set_error("mf_attention_fwd: 0 < L <= 512 required", -1);
  if (L > 256 && causal) return mf_set_error("mf_attention_fwd: causal masks need L <= 256", -1);
  if (ld_lse < L || (ld_qkv % 8) || (ld_out % 4)) return mf_set_error("mf_attention_fwd: bad strides", -1);
  const int LP = padded_len(L);
  hipStream_t st = (hipStream_t)stream;
  if (L > 256) {
    // register-resident scores at up to 512 keys: 8 waves (512 threads), 2 per SIMD, one workgroup per CU
    const int qs4 = attn_qsplit(N * H, L), tiles = (L + 15) / 16;
    const dim3 grid4(N * H, qs4), block4(64 * std::min(8, (tiles + qs4 - 1) / qs4));
#define CALLF4L(P) \
  attn_fwd4_kernel<P, false, 512><<<grid4, block4, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, L); break;
    switch (tiles * 16) {
      case 272: CALLF4L(272)
      case 288: CALLF4L(288)
      case 304: CALLF4L(304)
      case 320: CALLF4L(320)
      case 336: CALLF4L(336)
      case 352: CALLF4L(352)
      case 368: CALLF4L(368)
      case 384: CALLF4L(384)
      case 400: CALLF4L(400)
      case 416: CALLF4L(416)
      case 432: CALLF4L(432)
      case 448: CALLF4L(448)
      case 464: CALLF4L(464)
      case 480: CALLF4L(480)
      case 496: CALLF4L(496)
      case 512: CALLF4L(512)
      default: return mf_set_error("attention: bad padded length", -1);
    }
#undef CALLF4L
    MF_CHECK_LAUNCH();
    return 0;
  }
  // many heads of a long sequence (the eval engine's 400-image launches: 4 800 heads of 199 rows): the persistent
  // double-buffered kernel, one workgroup per CU walking ~19 heads (tests/diagnostics/attn_bench.py, r05:
  // 172.5 -> 148.8 us at 400 images, bit-identical; at 1 200 heads even, at c4's 384 heads 14.1 -> 17.3 us and at
  // the causal 77-row text heads 79 -> 83 us, so not there)
  if (N * H >= 2048 && L > 128) {
    const int tiles = (L + 15) / 16;
    const int LP16 = tiles * 16;
    const int per_cu = std::max(1, std::min((160 * 1024) / (512 * LP16), 16 / tiles));
    const int grid = std::min(N * H, mf_cu_count() * per_cu);
#define CALLFP(P)                                                                                                \
  if (causal)                                                                                                    \
    attn_fwdp_kernel<P, true><<<grid, 64 * tiles, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, N * H); \
  else                                                                                                           \
    attn_fwdp_kernel<P, false><<<grid, 64 * tiles, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, N * H);
    switch (LP16) {
      case 16: CALLFP(16); break;
      case 48: CALLFP(48); break;
      case 80: CALLFP(80); break;
      case 112: CALLFP(112); break;
      case 144: CALLFP(144); break;
      case 176: CALLFP(176); break;
      case 208: CALLFP(208); break;
      case 240: CALLFP(240); break;
      default: MF_ATTN_DISPATCH(LP, CALLFP)
    }
#undef CALLFP
    MF_CHECK_LAUNCH();
    return 0;
  }
  {
    // the head's 16-query tiles split evenly over its workgroups (no workgroup without a tile)
    const int Lq = L;
    const int qs4 = attn_qsplit(N * H, L), tiles = (L + 15) / 16;
    const int nw4 = std::min(16, (tiles + qs4 - 1) / qs4);
    const dim3 grid4(N * H, qs4), block4(64 * nw4);
    const int LP16 = tiles * 16;  // keys staged in 16-row tiles (LP16 % 32 == 16: a half last chunk)
#define CALLF4(P)                                                                                             \
  if (causal)                                                                                                 \
    attn_fwd4_kernel<P, true><<<grid4, block4, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, Lq); \
  else                                                                                                        \
    attn_fwd4_kernel<P, false><<<grid4, block4, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, Lq);
    switch (LP16) {
      case 16: CALLF4(16); break;
      case 48: CALLF4(48); break;
      case 80: CALLF4(80); break;
      case 112: CALLF4(112); break;
      case 144: CALLF4(144); break;
      case 176: CALLF4(176); break;
      case 208: CALLF4(208); break;
      case 240: CALLF4(240); break;
      default: MF_ATTN_DISPATCH(LP, CALLF4)
    }
#undef CALLF4
    MF_CHECK_LAUNCH();
    return 0;
  }
}

// The first q_rows query rows of every head only (K / V of all L rows): the forward-only engine's last vision block,
// whose output is read only at each image's class token (ln_post, clip/model.py:567), needs query row 0 of every
// head.  One workgroup per head, one wave per 16-query tile; each computed row is bit-identical to mf_attention_fwd's.
extern "C" int mf_attention_fwd_rows(const void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse,
                                     int ld_lse, int N, int L, int H, int causal, int q_rows, void* stream) {
  if (N <= 0) return 0;
  if (L <= 0 || L > 256) return mf_set_error("mf_attention_fwd_rows: 0 < L <= 256 required", -1);
  if (q_rows <= 0 || q_rows > L) return mf_set_error("mf_attention_fwd_rows: 0 < q_rows <= L required", -1);
  if (ld_lse < L || (ld_qkv % 8) || (ld_out % 4)) return mf_set_error("mf_attention_fwd_rows: bad strides", -1);
  const int LP = padded_len(L);
  hipStream_t st = (hipStream_t)stream;
  const int Lq = q_rows;
  const int tiles = (L + 15) / 16;
  const dim3 grid4(N * H, 1), block4(64 * ((q_rows + 15) / 16));
  const int LP16 = tiles * 16;
#define CALLF4(P)                                                                                             \
  if (causal)                                                                                                 \
    attn_fwd4_kernel<P, true><<<grid4, block4, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, Lq); \
  else                                                                                                        \
    attn_fwd4_kernel<P, false><<<grid4, block4, 0, st>>>((const f16*)qkv, ld_qkv, (f16*)out, ld_out, lse, ld_lse, L, H, Lq);
  switch (LP16) {
    case 16: CALLF4(16); break;
    case 48: CALLF4(48); break;
    case 80: CALLF4(80); break;
    case 112: CALLF4(112); break;
    case 144: CALLF4(144); break;
    case 176: CALLF4(176); break;
    case 208: CALLF4(208); break;
    case 240: CALLF4(240); break;
    default: MF_ATTN_DISPATCH(LP, CALLF4)
  }
#undef CALLF4
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_attention_bwd(const void* qkv, int64_t ld_qkv, const void* out, int64_t ld_out, const void* dout,
                                int64_t ld_dout, const float* lse, float* dq_dot_ws, int ld_lse, void* dqkv,
                                int64_t ld_dqkv, int N, int L, int H, int causal, void* stream) {
  if (N <= 0) return 0;
  if (L <= 0 || L > 512) return mf_set_error("mf_attention_bwd: 0 < L <= 512 required", -1);
  if (L > 256 && causal) return mf_set_error("mf_attention_bwd: causal masks need L <= 256", -1);
  if (ld_lse < L || (ld_qkv % 8) || (ld_dout % 8) || (ld_dqkv % 4)) return mf_set_error("mf_attention_bwd: bad strides", -1);
  const int LP = padded_len(L);
  hipStream_t st = (hipStream_t)stream;
  if (L > 256) {
    const int64_t tot = (int64_t)N * H * L;
    attn_bwd_dot_kernel<<<(tot + 255) / 256, 256, 0, st>>>((const f16*)out, ld_out, (const f16*)dout, ld_dout,
                                                          dq_dot_ws, ld_lse, N, L, H);
    MF_CHECK_LAUNCH();
    const dim3 grid(N * H, attn_qsplit(N * H, L)), block(attn_threads(L));
#define CALLBL(P)                                                                                                  \
  attn_bwd_dkv_kernel<P, false><<<grid, block, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)dout, ld_dout, lse,     \
                                                      dq_dot_ws, ld_lse, (f16*)dqkv, ld_dqkv, L, H);               \
  attn_bwd_dq_kernel<P, false><<<grid, block, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)dout, ld_dout, lse,      \
                                                     dq_dot_ws, ld_lse, (f16*)dqkv, ld_dqkv, L, H);
    MF_ATTN_DISPATCH_LONG(LP, CALLBL)
#undef CALLBL
    MF_CHECK_LAUNCH();
    return 0;
  }
  if (LP <= 224) {  // one fused workgroup per (sequence, head), 16 keys per wave
    const dim3 gridf(N * H), blockf(64 * (LP / 16));
#define CALLBF(P)                                                                                                  \
  if (causal)                                                                                                      \
    attn_bwd_fused_kernel<P, true, 1><<<gridf, blockf, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)out, ld_out,  \
                                                              (const f16*)dout, ld_dout, lse, ld_lse, (f16*)dqkv,   \
                                                              ld_dqkv, L, H);                                      \
  else                                                                                                             \
    attn_bwd_fused_kernel<P, false, 1><<<gridf, blockf, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)out, ld_out, \
                                                               (const f16*)dout, ld_dout, lse, ld_lse, (f16*)dqkv,  \
                                                               ld_dqkv, L, H);
    switch (LP) {
      case 32: CALLBF(32); break;
      case 64: CALLBF(64); break;
      case 96: CALLBF(96); break;
      case 128: CALLBF(128); break;
      case 160: CALLBF(160); break;
      case 192: CALLBF(192); break;
      case 224: CALLBF(224); break;
      default: return mf_set_error("attention: bad padded length", -1);
    }
#undef CALLBF
    MF_CHECK_LAUNCH();
    return 0;
  }
  const int64_t tot = (int64_t)N * H * L;
  attn_bwd_dot_kernel<<<(tot + 255) / 256, 256, 0, st>>>((const f16*)out, ld_out, (const f16*)dout, ld_dout,
                                                        dq_dot_ws, ld_lse, N, L, H);
  MF_CHECK_LAUNCH();
  const dim3 grid(N * H, attn_qsplit(N * H, L)), block(attn_threads(L));
#define CALLB(P)                                                                                                 \
  if (causal) {                                                                                                  \
    attn_bwd_dkv_kernel<P, true><<<grid, block, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)dout, ld_dout, lse,    \
                                                       dq_dot_ws, ld_lse, (f16*)dqkv, ld_dqkv, L, H);              \
    attn_bwd_dq_kernel<P, true><<<grid, block, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)dout, ld_dout, lse,     \
                                                      dq_dot_ws, ld_lse, (f16*)dqkv, ld_dqkv, L, H);               \
  } else {                                                                                                       \
    attn_bwd_dkv_kernel<P, false><<<grid, block, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)dout, ld_dout, lse,   \
                                                        dq_dot_ws, ld_lse, (f16*)dqkv, ld_dqkv, L, H);             \
    attn_bwd_dq_kernel<P, false><<<grid, block, 0, st>>>((const f16*)qkv, ld_qkv, (const f16*)dout, ld_dout, lse,    \
                                                       dq_dot_ws, ld_lse, (f16*)dqkv, ld_dqkv, L, H);              \
  }
  MF_ATTN_DISPATCH(LP, CALLB)
#undef CALLB
  MF_CHECK_LAUNCH();
  return 0;
}

// qkv = x W_in^T + b_in (fp16, bias epilogue) and out / lse = SDPA(qkv) in one launch (qkv_attn_fwd_kernel):
// the vision tower's blocks (D = 768, 193..208 tokens) and the text tower's (D = 512, causal, 65..80 tokens)
extern "C" int mf_qkv_attention_fwd(const void* x, int64_t ld_x, int x_rows, const void* w, const void* bias,
                                    void* qkv, int64_t ld_qkv, void* out, int64_t ld_out, float* lse, int ld_lse,
                                    int N, int L, int H, int causal, void* stream) {
  if (N <= 0) return 0;
  const int D = H * 64;
  if ((ld_x % 8) || (ld_qkv % 8) || (ld_out % 4) || ld_lse < L || ld_x < D || ld_qkv < 3 * D ||
      (uintptr_t)x % 16 || (uintptr_t)w % 16 || (uintptr_t)qkv % 16 || (uintptr_t)bias % 8)
    return mf_set_error("mf_qkv_attention_fwd: bad strides / alignment", -1);
  if (x_rows < N * L) return mf_set_error("mf_qkv_attention_fwd: x has fewer than N*L rows", -1);
  hipStream_t st = (hipStream_t)stream;
  if (D == 768 && !causal && L > 192 && L <= 208) {
    qkv_attn_fwd_vision_kernel<<<N * H, 896, 0, st>>>(
        (const f16*)x, ld_x, x_rows, (const f16*)w, (const f16*)bias, (f16*)qkv, ld_qkv, (f16*)out, ld_out, lse,
        ld_lse, L, H);
  } else if (D == 512 && causal && L > 64 && L <= 80) {
    qkv_attn_fwd_text_kernel<<<N * H, 384, 0, st>>>(
        (const f16*)x, ld_x, x_rows, (const f16*)w, (const f16*)bias, (f16*)qkv, ld_qkv, (f16*)out, ld_out, lse,
        ld_lse, L, H);
  } else {
    return mf_set_error("mf_qkv_attention_fwd: shape outside the fused kernels (vision D=768 L 193..208, text "
                        "D=512 causal L 65..80)", -1);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_qkv_attention_supported(int N, int L, int H, int causal) {
  const int D = H * 64;
  return N > 0 && ((D == 768 && !causal && L > 192 && L <= 208) || (D == 512 && causal && L > 64 && L <= 80));
}
