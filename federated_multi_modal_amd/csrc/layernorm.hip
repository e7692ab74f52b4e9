// LayerNorm forward/backward for CLIP's fp16 LayerNorm subclass (clip/model.py:153-159):
// fp16 rows in, statistics and affine math in fp32, fp16 out; gamma/beta are fp32 and trainable
// everywhere (trainers/maple.py:451-454), so the backward also produces dgamma/dbeta.
//
// HBM-bound: 2 B read + 2 B write per element forward, ~6 B per element backward.  One wave per
// row, 8-byte (4 x fp16) vector accesses, statistics by wave64 shuffles.  An optional int32 row
// index gathers rows (ln_post on each image's class token, ln_final on each prompt's EOT token,
// clip/model.py:567 and trainers/maple.py:72-76).  dgamma/dbeta are reduced deterministically:
// per-block partial sums, then a column reduction (no float atomics).
#include <cstdlib>

#include "mf_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int LN_WAVES = 4;
constexpr int LN_ROWS_PER_BLOCK = 16;

// y = ((x*rstd) + (-rstd*mean)) * gamma + beta, the operation order of torch's CPU kernel
template <int D>
__global__ __launch_bounds__(256) void ln_fwd_kernel(const f16* __restrict__ x, int64_t ldx,
                                                    const int* __restrict__ ridx, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, f16* __restrict__ y,
                                                    int64_t ldy, float* __restrict__ mean_out,
                                                    float* __restrict__ rstd_out, int rows) {
  constexpr int CH = D / 256;  // vec4 chunks per lane
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * LN_WAVES + (threadIdx.x >> 6);
  if (row >= rows) return;
  const int src = ridx ? ridx[row] : row;
  const f16* xr = x + (int64_t)src * ldx;
  float v[CH * 4];
  float s = 0.f;
#pragma unroll
  for (int cnt = 0; cnt < CH; ++cnt) {
    const int c = lane + 64 * cnt;
    f16x4 t = *(const f16x4*)(xr + 4 * c);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[cnt * 4 + e] = (float)t[e];
      s += v[cnt * 4 + e];
    }
  }
  const float mean = wave_sum(s) / (float)D;
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < CH * 4; ++i) {
    float d = v[i] - mean;
    ss += d * d;
  }
  const float var = wave_sum(ss) / (float)D;
  const float rstd = 1.0f / sqrtf(fmaxf(var, 0.f) + 1e-5f);
  const float bias = -rstd * mean;
  f16* yr = y + (int64_t)row * ldy;
#pragma unroll
  for (int cnt = 0; cnt < CH; ++cnt) {
    const int c = lane + 64 * cnt;
    f32x4 g = *(const f32x4*)(gamma + 4 * c);
    f32x4 b = *(const f32x4*)(beta + 4 * c);
    f16x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float t = v[cnt * 4 + e] * rstd;
      t = t + bias;
      t = t * g[e];
      t = t + b[e];
      o[e] = (f16)t;
    }
    *(f16x4*)(yr + 4 * c) = o;
  }
  if (lane == 0) {
    if (mean_out) mean_out[row] = mean;
    if (rstd_out) rstd_out[row] = rstd;
  }
}

// dx = rstd*(dy*g) + b*x + c with  b = (sum(dy*g)*mean - sum(dy*g*x)) * rstd^3 / D,
// c = -b*mean - sum(dy*g)*rstd/D   (fp32), then dx16 = fp16(dx) and, when a residual gradient
// is given, out = fp16(dres + dx16)  (the autograd accumulation of the two uses of x).
template <int D>
__global__ __launch_bounds__(256) void ln_bwd_kernel(const f16* __restrict__ dy, int64_t lddy,
                                                    const f16* __restrict__ x, int64_t ldx,
                                                    const int* __restrict__ ridx, const float* __restrict__ gamma,
                                                    const float* __restrict__ mean_in,
                                                    const float* __restrict__ rstd_in, const f16* dres,
                                                    int64_t ldres, f16* dx, int64_t lddx,
                                                    float* __restrict__ dg_part, float* __restrict__ db_part,
                                                    int rows) {
  constexpr int CH = D / 256;
  __shared__ float red_g[LN_WAVES][D];
  __shared__ float red_b[LN_WAVES][D];
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  float accg[CH * 4], accb[CH * 4];
#pragma unroll
  for (int i = 0; i < CH * 4; ++i) accg[i] = accb[i] = 0.f;
  const int r0 = blockIdx.x * LN_ROWS_PER_BLOCK;
  for (int rr = w; rr < LN_ROWS_PER_BLOCK; rr += LN_WAVES) {
    const int row = r0 + rr;
    if (row >= rows) break;
    const int src = ridx ? ridx[row] : row;
    const f16* xr = x + (int64_t)src * ldx;
    const f16* dyr = dy + (int64_t)row * lddy;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xv[CH * 4], dv[CH * 4], gv[CH * 4];
    float sdg = 0.f, sdgx = 0.f;
#pragma unroll
    for (int cnt = 0; cnt < CH; ++cnt) {
      const int c = lane + 64 * cnt;
      f16x4 tx = *(const f16x4*)(xr + 4 * c);
      f16x4 td = *(const f16x4*)(dyr + 4 * c);
      f32x4 g = *(const f32x4*)(gamma + 4 * c);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xv[cnt * 4 + e] = (float)tx[e];
        dv[cnt * 4 + e] = (float)td[e];
        gv[cnt * 4 + e] = g[e];
        float dg = dv[cnt * 4 + e] * g[e];
        sdg += dg;
        sdgx += dg * xv[cnt * 4 + e];
        float xhat = (xv[cnt * 4 + e] - mean) * rstd;
        accg[cnt * 4 + e] += dv[cnt * 4 + e] * xhat;
        accb[cnt * 4 + e] += dv[cnt * 4 + e];
      }
    }
    sdg = wave_sum(sdg);
    sdgx = wave_sum(sdgx);
    const float invD = 1.0f / (float)D;
    const float b = (sdg * mean - sdgx) * rstd * rstd * rstd * invD;
    const float c = -b * mean - sdg * rstd * invD;
    f16* dxr = dx + (int64_t)src * lddx;
    const f16* drr = dres ? dres + (int64_t)src * ldres : nullptr;
#pragma unroll
    for (int cnt = 0; cnt < CH; ++cnt) {
      const int cc = lane + 64 * cnt;
      f16x4 o;
      f16x4 rv;
      if (drr) rv = *(const f16x4*)(drr + 4 * cc);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float t = ((rstd * dv[cnt * 4 + e]) * gv[cnt * 4 + e] + b * xv[cnt * 4 + e]) + c;
        float t16 = r16(t);
        o[e] = drr ? (f16)((float)rv[e] + t16) : (f16)t16;
      }
      *(f16x4*)(dxr + 4 * cc) = o;
    }
  }
  // reduce the 4 waves' column partials through LDS
#pragma unroll
  for (int cnt = 0; cnt < CH; ++cnt) {
    const int c = lane + 64 * cnt;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      red_g[w][4 * c + e] = accg[cnt * 4 + e];
      red_b[w][4 * c + e] = accb[cnt * 4 + e];
    }
  }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += 256) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < LN_WAVES; ++k) {
      sg += red_g[k][col];
      sb += red_b[k][col];
    }
    dg_part[(int64_t)blockIdx.x * D + col] = sg;
    db_part[(int64_t)blockIdx.x * D + col] = sb;
  }
}

// ---- half-wave-per-row variants: 32 lanes own a row, 16-byte (8 x fp16) accesses, statistics by
// 32-lane butterflies.  The forward puts 8 rows in flight per 256-thread block; the backward gives
// every half-wave two rows whose loads are all issued before either is reduced.
MF_DEV float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int D, int RPH = 1>
__global__ __launch_bounds__(256) void ln_fwd2_kernel(const f16* __restrict__ x, int64_t ldx,
                                                     const int* __restrict__ ridx, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, f16* __restrict__ y,
                                                     int64_t ldy, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, int rows,
                                                     const float* __restrict__ inj = nullptr, int inj_L = 1,
                                                     int inj_row0 = 0, int inj_n = 0) {
  // RPH rows per half-wave (consecutive rows, every row's loads issued before the first is reduced): the
  // same per-row arithmetic with 1/RPH of the workgroups -- for the text tower, whose LayerNorms run beside
  // the vision tower and should hold as few CUs as possible (no injection: RPH = 1 there)
  static_assert(RPH == 1 || RPH == 2 || RPH == 4, "rows per half-wave");
  constexpr int CH = D / 256;  // 16-byte chunks per lane
  const int hl = threadIdx.x & 31;
  const int row0 = (blockIdx.x * 8 + (threadIdx.x >> 5)) * RPH;
  if (row0 >= rows) return;  // whole half-waves leave together: the butterflies stay within a half
  f16x8 t[RPH][CH];
#pragma unroll
  for (int r = 0; r < RPH; ++r) {
    const int row = row0 + r < rows ? row0 + r : row0;  // a past-the-end row re-reads row0, stores nothing
    const int src = ridx ? ridx[row] : row;
    const f16* xr = x + (int64_t)src * ldx;
    // deep-prompt injection fused in (inj != null, no ridx): rows inj_row0 .. inj_row0+inj_n-1 of every
    // inj_L-row sequence take fp16(prompt row) -- written back to x as mf_prompt_inject_fwd would -- and
    // are normalised from those values
    const int pr = inj ? row % inj_L - inj_row0 : -1;
    if (pr >= 0 && pr < inj_n) {
      const float* prow = inj + (int64_t)pr * D;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int c = 8 * (hl + 32 * j);
#pragma unroll
        for (int e = 0; e < 8; ++e) t[r][j][e] = (f16)prow[c + e];
        *(f16x8*)(const_cast<f16*>(xr) + c) = t[r][j];
      }
    } else {
#pragma unroll
      for (int j = 0; j < CH; ++j) t[r][j] = *(const f16x8*)(xr + 8 * (hl + 32 * j));
    }
  }
#pragma unroll
  for (int r = 0; r < RPH; ++r) {
    const int row = row0 + r;
    if (row >= rows) break;
    float v[CH * 8];
    // Reduction order identical to ln_fwd_kernel's: a 16-byte chunk holds the 4-element groups of two
    // of its lanes (2*hl and 2*hl+1); keep them as two partials, butterfly each over the half-wave
    // (= that kernel's xor 32..2 steps) and add them last (= its xor-1 step).
    float s0 = 0.f, s1 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        v[j * 8 + e] = (float)t[r][j][e];
        if (e < 4) s0 += v[j * 8 + e];
        else s1 += v[j * 8 + e];
      }
    const float mean = (half_sum(s0) + half_sum(s1)) / (float)D;
    float ss0 = 0.f, ss1 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = v[j * 8 + e] - mean;
        if (e < 4) ss0 += d * d;
        else ss1 += d * d;
      }
    const float var = (half_sum(ss0) + half_sum(ss1)) / (float)D;
    const float rstd = 1.0f / sqrtf(fmaxf(var, 0.f) + 1e-5f);
    const float bias = -rstd * mean;
    f16* yr = y + (int64_t)row * ldy;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = 8 * (hl + 32 * j);
      const f32x4 g0 = *(const f32x4*)(gamma + c), g1 = *(const f32x4*)(gamma + c + 4);
      const f32x4 b0 = *(const f32x4*)(beta + c), b1 = *(const f32x4*)(beta + c + 4);
      f16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float tt = v[j * 8 + e] * rstd;
        tt = tt + bias;
        tt = tt * (e < 4 ? g0[e] : g1[e - 4]);
        tt = tt + (e < 4 ? b0[e] : b1[e - 4]);
        o[e] = (f16)tt;
      }
      *(f16x8*)(yr + c) = o;
    }
    if (hl == 0) {
      if (mean_out) mean_out[row] = mean;
      if (rstd_out) rstd_out[row] = rstd;
    }
  }
}

// HWB half-waves per 16-row block: 8 (two rows each) or, for few blocks (ln_bwd_wide: below 256, i.e. the c4 text
// tower and the small clients), 16 (one row each: twice the waves in flight per row block).  The partials stay bit-identical: a pair of
// one-row half-waves is summed first (fl(a + b) = fl(b + a), and 0 + a is exact), which is what a two-row
// half-wave's accumulator holds, then the 8 pair sums in order.
template <int D, int HWB = 8, bool LIVE = false>
__global__ __launch_bounds__(HWB * 32) void ln_bwd2_kernel(const f16* __restrict__ dy, int64_t lddy,
                                                     const f16* __restrict__ x, int64_t ldx,
                                                     const int* __restrict__ ridx, const float* __restrict__ gamma,
                                                     const float* __restrict__ mean_in,
                                                     const float* __restrict__ rstd_in, const f16* dres,
                                                     int64_t ldres, f16* dx, int64_t lddx,
                                                     float* __restrict__ dg_part, float* __restrict__ db_part,
                                                     int rows, float* __restrict__ inj_part = nullptr,
                                                     int inj_L = 1, int inj_row0 = 0, int inj_n = 0,
                                                     int seg_live = 0, int seg_full = 0) {
  // LIVE: `rows` counts VIRTUAL rows of seg_full-row sequences, of which the first seg_live of each are stored
  // (compact row (v / seg_full) * seg_live + v % seg_full); the rest are rows whose dy is exactly zero (the text
  // tower's tokens after every class's EOT, mf_layernorm_bwd_live): they add nothing, so the row blocks, and with
  // them the dgamma / dbeta partials, are those of the full-length tower.  A dead row's loads still run (from
  // compact row 0, a cache hit) so that the load / wait structure is the plain kernel's.  (r05 saw a version that
  // branched around them give run-to-run different dgamma partials under tower concurrency; r06 traced that to the
  // packed fp32 VALU path, which the library no longer builds with -- DESIGN.md §6, tests/test_isa.py.)
  constexpr int CH = D / 256;
  static_assert(HWB == 8 || HWB == 16, "half-waves per block");
  constexpr int RPH = LN_ROWS_PER_BLOCK / HWB;  // rows per half-wave
  __shared__ float red_g[HWB][D];
  __shared__ float red_b[HWB][D];
  const int hl = threadIdx.x & 31;
  const int hw = threadIdx.x >> 5;
  float gv[CH * 8];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const f32x4 g0 = *(const f32x4*)(gamma + 8 * (hl + 32 * j)), g1 = *(const f32x4*)(gamma + 8 * (hl + 32 * j) + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      gv[j * 8 + e] = g0[e];
      gv[j * 8 + 4 + e] = g1[e];
    }
  }
  float accg[CH * 8], accb[CH * 8];
#pragma unroll
  for (int i = 0; i < CH * 8; ++i) accg[i] = accb[i] = 0.f;
  // every load of the half-wave's rows first (rows past the end clamp to a valid row and are skipped)
  const int r0 = blockIdx.x * LN_ROWS_PER_BLOCK + hw * RPH;
  f16x8 tx[RPH][CH], td[RPH][CH], tr[RPH][CH];
  int srcs[RPH];
  bool use[RPH];
  float means[RPH], rstds[RPH];
#pragma unroll
  for (int k = 0; k < RPH; ++k) {
    int row = min(r0 + k, rows - 1);
    use[k] = r0 + k < rows;
    if constexpr (LIVE) {
      const int t = row % seg_full;
      use[k] = use[k] && t < seg_live;
      row = use[k] ? (row / seg_full) * seg_live + t : 0;
    }
    srcs[k] = ridx ? ridx[row] : row;
    means[k] = mean_in[row];
    rstds[k] = rstd_in[row];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = 8 * (hl + 32 * j);
      tx[k][j] = *(const f16x8*)(x + (int64_t)srcs[k] * ldx + c);
      td[k][j] = *(const f16x8*)(dy + (int64_t)row * lddy + c);
      if (dres) tr[k][j] = *(const f16x8*)(dres + (int64_t)srcs[k] * ldres + c);
    }
  }
#pragma unroll
  for (int k = 0; k < RPH; ++k) {
    if (use[k]) {
      const float mean = means[k], rstd = rstds[k];
      float sdg0 = 0.f, sdg1 = 0.f, sdgx0 = 0.f, sdgx1 = 0.f;  // ln_bwd_kernel's order (see ln_fwd2_kernel)
#pragma unroll
      for (int j = 0; j < CH; ++j)
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float xv = (float)tx[k][j][e], dv = (float)td[k][j][e];
          const float dg = dv * gv[j * 8 + e];
          if (e < 4) {
            sdg0 += dg;
            sdgx0 += dg * xv;
          } else {
            sdg1 += dg;
            sdgx1 += dg * xv;
          }
          const float xhat = (xv - mean) * rstd;
          accg[j * 8 + e] += dv * xhat;
          accb[j * 8 + e] += dv;
        }
      const float sdg = half_sum(sdg0) + half_sum(sdg1);
      const float sdgx = half_sum(sdgx0) + half_sum(sdgx1);
      const float invD = 1.0f / (float)D;
      const float b = (sdg * mean - sdgx) * rstd * rstd * rstd * invD;
      const float c = -b * mean - sdg * rstd * invD;
      f16* dxr = dx + (int64_t)srcs[k] * lddx;
      // injected deep-prompt rows (inj_part != null, no ridx): their gradient goes to the prompt, not to
      // the previous layer -- the fp16 value is kept as an fp32 partial [sequence][prompt row][D] (summed
      // over sequences by the deferred column reduction) and the dx row is zeroed
      const int pr = inj_part ? srcs[k] % inj_L - inj_row0 : -1;
      float* ipr = (pr >= 0 && pr < inj_n) ? inj_part + ((int64_t)(srcs[k] / inj_L) * inj_n + pr) * D : nullptr;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = ((rstd * (float)td[k][j][e]) * gv[j * 8 + e] + b * (float)tx[k][j][e]) + c;
          const float t16 = r16(t);
          o[e] = dres ? (f16)((float)tr[k][j][e] + t16) : (f16)t16;
        }
        if (ipr) {
          const int cc = 8 * (hl + 32 * j);
          *(f32x4*)(ipr + cc) = (f32x4){(float)o[0], (float)o[1], (float)o[2], (float)o[3]};
          *(f32x4*)(ipr + cc + 4) = (f32x4){(float)o[4], (float)o[5], (float)o[6], (float)o[7]};
          o = f16x8{};
        }
        *(f16x8*)(dxr + 8 * (hl + 32 * j)) = o;
      }
    }
  }
  // the half-waves' column partials through LDS (fixed order: deterministic)
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red_g[hw][8 * (hl + 32 * j) + e] = accg[j * 8 + e];
      red_b[hw][8 * (hl + 32 * j) + e] = accb[j * 8 + e];
    }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += HWB * 32) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (HWB == 16) {
        sg += red_g[2 * k][col] + red_g[2 * k + 1][col];
        sb += red_b[2 * k][col] + red_b[2 * k + 1][col];
      } else {
        sg += red_g[k][col];
        sb += red_b[k][col];
      }
    }
    dg_part[(int64_t)blockIdx.x * D + col] = sg;
    db_part[(int64_t)blockIdx.x * D + col] = sb;
  }
}

// one row per half-wave (16 half-waves per row block) when the row blocks alone cannot fill the chip: below 256
// blocks (the c4 text tower's 183, the small clients' ~50; tests/diagnostics/ln_bench.py, r04: 8.43 -> 7.58 us at
// 2 926 x 512, 8.11 -> 7.43 at 796 x 768; at 6 368 x 768, 398 blocks, 14.3 -> 15.7, so not there).  Both forms
// produce bit-identical partials (measured r04); tests/test_kernels_gpu.py::test_layernorm covers both regimes.
inline bool ln_bwd_wide(int nblk) { return nblk < 256; }

}  // namespace

extern "C" int mf_layernorm_fwd(const void* x, int64_t ldx, const int* row_index, const float* gamma,
                                const float* beta, void* y, int64_t ldy, float* mean, float* rstd, int rows, int D,
                                void* stream) {
  if (rows <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool v16 = ((uintptr_t)x % 16 == 0) && ((uintptr_t)y % 16 == 0) && (ldx % 8 == 0) && (ldy % 8 == 0);
  // 16-byte accesses, one row per half-wave (the wave-per-row kernels below take unaligned rows)
  if (v16 && (D == 768 || D == 512)) {
    const dim3 g2((rows + 7) / 8);
    if (D == 768)
      ln_fwd2_kernel<768><<<g2, 256, 0, st>>>((const f16*)x, ldx, row_index, gamma, beta, (f16*)y, ldy, mean, rstd, rows);
    else
      ln_fwd2_kernel<512><<<g2, 256, 0, st>>>((const f16*)x, ldx, row_index, gamma, beta, (f16*)y, ldy, mean, rstd, rows);
    MF_CHECK_LAUNCH();
    return 0;
  }
  dim3 grid((rows + LN_WAVES - 1) / LN_WAVES);
  if (D == 768)
    ln_fwd_kernel<768><<<grid, 256, 0, st>>>((const f16*)x, ldx, row_index, gamma, beta, (f16*)y, ldy, mean, rstd, rows);
  else if (D == 512)
    ln_fwd_kernel<512><<<grid, 256, 0, st>>>((const f16*)x, ldx, row_index, gamma, beta, (f16*)y, ldy, mean, rstd, rows);
  else
    return mf_set_error("mf_layernorm_fwd: D must be 512 or 768", -1);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_layernorm_bwd_blocks(int rows) { return (rows + LN_ROWS_PER_BLOCK - 1) / LN_ROWS_PER_BLOCK; }

extern "C" int mf_layernorm_bwd(const void* dy, int64_t lddy, const void* x, int64_t ldx, const int* row_index,
                                const float* gamma, const float* mean, const float* rstd, const void* dres,
                                int64_t ldres, void* dx, int64_t lddx, float* dgamma, float* dbeta, float* workspace,
                                int rows, int D, int accumulate, void* stream) {
  if (rows <= 0) return 0;
  if (D != 512 && D != 768) return mf_set_error("mf_layernorm_bwd: D must be 512 or 768", -1);
  const int nblk = mf_layernorm_bwd_blocks(rows);
  float* dg_part = workspace;
  float* db_part = workspace + (int64_t)nblk * D;
  hipStream_t st = (hipStream_t)stream;
  const bool v16 = ((uintptr_t)dy % 16 == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)dx % 16 == 0) &&
                   (!dres || ((uintptr_t)dres % 16 == 0 && ldres % 8 == 0)) && lddy % 8 == 0 && ldx % 8 == 0 &&
                   lddx % 8 == 0;
  if (v16) {
    if (D == 768 && ln_bwd_wide(nblk))
      ln_bwd2_kernel<768, 16><<<nblk, 512, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, row_index, gamma, mean,
                                                    rstd, (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows);
    else if (D == 768)
      ln_bwd2_kernel<768><<<nblk, 256, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, row_index, gamma, mean, rstd,
                                                (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows);
    else if (ln_bwd_wide(nblk))
      ln_bwd2_kernel<512, 16><<<nblk, 512, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, row_index, gamma, mean,
                                                    rstd, (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows);
    else
      ln_bwd2_kernel<512><<<nblk, 256, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, row_index, gamma, mean, rstd,
                                                (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows);
  } else if (D == 768)
    ln_bwd_kernel<768><<<nblk, 256, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, row_index, gamma, mean, rstd,
                                             (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows);
  else
    ln_bwd_kernel<512><<<nblk, 256, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, row_index, gamma, mean, rstd,
                                             (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows);
  MF_CHECK_LAUNCH();
  if (!dgamma && !dbeta) return 0;  // partials only: the caller reduces them later (mf_col_reduce_batch)
  if (!dgamma || !dbeta) return mf_set_error("mf_layernorm_bwd: dgamma and dbeta go together", -1);
  col_reduce_kernel<false><<<dim3((D + 63) / 64, 2), 1024, 0, st>>>(dg_part, db_part, nblk, D, D, dgamma, dbeta,
                                                                    accumulate);
  MF_CHECK_LAUNCH();
  return 0;
}

// ---- batched deferred column reductions (every LayerNorm's dgamma/dbeta of a backward pass in one launch)
namespace {
struct ColReduceDesc {
  const float* part;  // [nblk][C] partial sums
  float* out;         // [C]
  int nblk, C, accumulate, pad;
};
__global__ __launch_bounds__(1024) void col_reduce_batch_kernel(const ColReduceDesc* __restrict__ descs) {
  __shared__ float red[16][65];
  const ColReduceDesc d = descs[blockIdx.y];
  if ((int)blockIdx.x * 64 >= d.C) return;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < d.C) {
    int b = g;
    for (; b + 48 < d.nblk; b += 64) {
      s0 += d.part[(int64_t)b * d.C + c];
      s1 += d.part[(int64_t)(b + 16) * d.C + c];
      s2 += d.part[(int64_t)(b + 32) * d.C + c];
      s3 += d.part[(int64_t)(b + 48) * d.C + c];
    }
    for (; b < d.nblk; b += 16) s0 += d.part[(int64_t)b * d.C + c];
  }
  red[g][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && c < d.C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][lane];
    d.out[c] = d.accumulate ? d.out[c] + s : s;
  }
}
}  // namespace

extern "C" int mf_col_reduce_desc_bytes(void) { return (int)sizeof(ColReduceDesc); }

extern "C" int mf_col_reduce_batch(const void* descs, int n, int max_cols, void* stream) {
  if (n <= 0) return 0;
  col_reduce_batch_kernel<<<dim3((max_cols + 63) / 64, n), 1024, 0, (hipStream_t)stream>>>(
      (const ColReduceDesc*)descs);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_prompt_inject_fwd(void* x, const float* prompt, int N, int L, int row0, int nrows, int D,
                                    void* stream);

// LayerNorm with the deep-prompt injection of the same rows fused in: equivalent (bit for bit) to
// mf_prompt_inject_fwd(x, prompt, rows / L, L, row0, nrows, D) followed by mf_layernorm_fwd on x
// (clip/model.py:320-349 injection at the start of a block, then its ln_1).
extern "C" int mf_layernorm_fwd_inject(void* x, int64_t ldx, const float* gamma, const float* beta, void* y,
                                       int64_t ldy, float* mean, float* rstd, int rows, int D, const float* prompt,
                                       int L, int row0, int nrows, void* stream) {
  if (rows <= 0) return 0;
  if (L <= 0 || rows % L || row0 < 0 || row0 + nrows > L) return mf_set_error("mf_layernorm_fwd_inject: rows", -1);
  hipStream_t st = (hipStream_t)stream;
  const bool v16 = ((uintptr_t)x % 16 == 0) && ((uintptr_t)y % 16 == 0) && (ldx % 8 == 0) && (ldy % 8 == 0);
  if (ldx != D || !(v16 && (D == 768 || D == 512))) {
    const int rc = mf_prompt_inject_fwd(x, prompt, rows / L, L, row0, nrows, D, stream);
    return rc ? rc : mf_layernorm_fwd(x, ldx, nullptr, gamma, beta, y, ldy, mean, rstd, rows, D, stream);
  }
  const dim3 g2((rows + 7) / 8);
  if (D == 768)
    ln_fwd2_kernel<768><<<g2, 256, 0, st>>>((const f16*)x, ldx, nullptr, gamma, beta, (f16*)y, ldy, mean, rstd, rows,
                                            prompt, L, row0, nrows);
  else
    ln_fwd2_kernel<512><<<g2, 256, 0, st>>>((const f16*)x, ldx, nullptr, gamma, beta, (f16*)y, ldy, mean, rstd, rows,
                                            prompt, L, row0, nrows);
  MF_CHECK_LAUNCH();
  return 0;
}

// LayerNorm backward (partials only, as mf_layernorm_bwd with dgamma = dbeta = NULL) with the deep-prompt
// injection backward of the same rows fused in: rows row0 .. row0+nrows-1 of every L-row sequence
// write their dx value as an fp32 partial inj_part[n][r][D] (the prompt gradient is their sum over n,
// left to the caller's mf_col_reduce_batch with nblk = rows / L, C = nrows * D) and a zero dx row.
// Replaces mf_layernorm_bwd + mf_prompt_inject_bwd(zero_rows) (clip/model.py:153-159, 320-349).
extern "C" int mf_layernorm_bwd_inject(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* gamma,
                                       const float* mean, const float* rstd, const void* dres, int64_t ldres,
                                       void* dx, int64_t lddx, float* workspace, int rows, int D, float* inj_part,
                                       int L, int row0, int nrows, void* stream) {
  if (rows <= 0) return 0;
  if (D != 512 && D != 768) return mf_set_error("mf_layernorm_bwd_inject: D must be 512 or 768", -1);
  if (L <= 0 || rows % L || row0 < 0 || row0 + nrows > L) return mf_set_error("mf_layernorm_bwd_inject: rows", -1);
  const bool v16 = ((uintptr_t)dy % 16 == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)dx % 16 == 0) &&
                   (!dres || ((uintptr_t)dres % 16 == 0 && ldres % 8 == 0)) && lddy % 8 == 0 && ldx % 8 == 0 &&
                   lddx % 8 == 0 && (uintptr_t)inj_part % 16 == 0;
  if (!v16) return mf_set_error("mf_layernorm_bwd_inject: needs 16-byte aligned rows", -1);
  const int nblk = mf_layernorm_bwd_blocks(rows);
  float* dg_part = workspace;
  float* db_part = workspace + (int64_t)nblk * D;
  hipStream_t st = (hipStream_t)stream;
  if (D == 768 && ln_bwd_wide(nblk))
    ln_bwd2_kernel<768, 16><<<nblk, 512, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, nullptr, gamma, mean, rstd,
                                                  (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows,
                                                  inj_part, L, row0, nrows);
  else if (D == 768)
    ln_bwd2_kernel<768><<<nblk, 256, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, nullptr, gamma, mean, rstd,
                                              (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows, inj_part,
                                              L, row0, nrows);
  else if (ln_bwd_wide(nblk))
    ln_bwd2_kernel<512, 16><<<nblk, 512, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, nullptr, gamma, mean, rstd,
                                                  (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows,
                                                  inj_part, L, row0, nrows);
  else
    ln_bwd2_kernel<512><<<nblk, 256, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, nullptr, gamma, mean, rstd,
                                              (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows, inj_part,
                                              L, row0, nrows);
  MF_CHECK_LAUNCH();
  return 0;
}

// LayerNorm backward (partials only) of a tower that stores only the first L_live rows of each of its `seqs`
// L_full-row sequences (the EOT-truncated text tower: rows past every class's EOT have exactly zero gradient and
// are not computed).  The compact rows (seqs * L_live, row n * L_live + t) are processed as the rows t < L_live of
// the full-length tower: the row blocks, the block partials (workspace: 2 * mf_layernorm_bwd_blocks(seqs * L_full)
// * D floats) and so the dgamma / dbeta that mf_col_reduce_batch forms from them are bit for bit those of
// mf_layernorm_bwd over the full tower, whose extra rows add zeros.  inj_part (optional): the deep-prompt
// injection backward of mf_layernorm_bwd_inject, rows row0 .. row0 + nrows - 1 of each sequence.
extern "C" int mf_layernorm_bwd_live(const void* dy, int64_t lddy, const void* x, int64_t ldx, const float* gamma,
                                     const float* mean, const float* rstd, const void* dres, int64_t ldres, void* dx,
                                     int64_t lddx, float* workspace, int seqs, int L_live, int L_full, int D,
                                     float* inj_part, int row0, int nrows, void* stream) {
  if (seqs <= 0) return 0;
  if (D != 512 && D != 768) return mf_set_error("mf_layernorm_bwd_live: D must be 512 or 768", -1);
  if (L_live <= 0 || L_live > L_full) return mf_set_error("mf_layernorm_bwd_live: 0 < L_live <= L_full", -1);
  if (inj_part && (row0 < 0 || row0 + nrows > L_live)) return mf_set_error("mf_layernorm_bwd_live: prompt rows", -1);
  const bool v16 = ((uintptr_t)dy % 16 == 0) && ((uintptr_t)x % 16 == 0) && ((uintptr_t)dx % 16 == 0) &&
                   (!dres || ((uintptr_t)dres % 16 == 0 && ldres % 8 == 0)) && lddy % 8 == 0 && ldx % 8 == 0 &&
                   lddx % 8 == 0 && (uintptr_t)inj_part % 16 == 0;
  if (!v16) return mf_set_error("mf_layernorm_bwd_live: needs 16-byte aligned rows", -1);
  const int rows = seqs * L_full;  // virtual
  const int nblk = mf_layernorm_bwd_blocks(rows);
  float* dg_part = workspace;
  float* db_part = workspace + (int64_t)nblk * D;
  const int inj_n = inj_part ? nrows : 0;
  hipStream_t st = (hipStream_t)stream;
#define MF_LN_LIVE(DD, HW, TH)                                                                                       \
  ln_bwd2_kernel<DD, HW, true><<<nblk, TH, 0, st>>>((const f16*)dy, lddy, (const f16*)x, ldx, nullptr, gamma, mean, rstd, \
                                              (const f16*)dres, ldres, (f16*)dx, lddx, dg_part, db_part, rows,     \
                                              inj_part, L_live, row0, inj_n, L_live, L_full)
  if (D == 768 && ln_bwd_wide(nblk)) MF_LN_LIVE(768, 16, 512);
  else if (D == 768) MF_LN_LIVE(768, 8, 256);
  else if (ln_bwd_wide(nblk)) MF_LN_LIVE(512, 16, 512);
  else MF_LN_LIVE(512, 8, 256);
#undef MF_LN_LIVE
  MF_CHECK_LAUNCH();
  return 0;
}
