// Diagnostic (GPU box): where does ln_bwd2_kernel<768, 8> (csrc/layernorm.hip) spend its time at the c4 vision
// shape (6 368 rows)?  A copy of its arithmetic with parts switched off by MODE bits (timing only; the outputs of
// MODE != 0 are not LayerNorm gradients):
//   1: gamma not loaded (gv = 1)          2: no LDS column reduction / partial stores
//   4: no dx stores                        8: no dres loads (the residual-gradient operand)
//  16: dx stored non-temporally           64: dx = x + dy + dres only (the same loads / stores, no LayerNorm)
// Built by run.py with hipcc into this directory; nothing here is part of libmapfed.so.
#include <hip/hip_runtime.h>
#include <cstdint>

typedef _Float16 f16;
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#pragma clang fp contract(off)

namespace {
__device__ __forceinline__ float half_sum(float v) {
#pragma unroll
  for (int o = 16; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float r16(float v) { return (float)(f16)v; }

template <int MODE>
__global__ __launch_bounds__(256) void lnb_kernel(const f16* __restrict__ dy, const f16* __restrict__ x,
                                                  const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                  const float* __restrict__ rstd_in, const f16* __restrict__ dres,
                                                  f16* __restrict__ dx, float* __restrict__ dg_part,
                                                  float* __restrict__ db_part, int rows) {
  constexpr int D = 768, CH = 3, HWB = 8, RPH = 2;
  __shared__ float red_g[HWB][D];
  __shared__ float red_b[HWB][D];
  const int hl = threadIdx.x & 31, hw = threadIdx.x >> 5;
  float gv[CH * 8];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    if (MODE & 1) {
#pragma unroll
      for (int e = 0; e < 8; ++e) gv[j * 8 + e] = 1.f;
    } else {
      const f32x4 g0 = *(const f32x4*)(gamma + 8 * (hl + 32 * j)), g1 = *(const f32x4*)(gamma + 8 * (hl + 32 * j) + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        gv[j * 8 + e] = g0[e];
        gv[j * 8 + 4 + e] = g1[e];
      }
    }
  }
  float accg[CH * 8], accb[CH * 8];
#pragma unroll
  for (int i = 0; i < CH * 8; ++i) accg[i] = accb[i] = 0.f;
  const int r0 = blockIdx.x * 16 + hw * RPH;
  f16x8 tx[RPH][CH], td[RPH][CH], tr[RPH][CH];
  if (MODE & 64) {
#pragma unroll
    for (int k = 0; k < RPH; ++k) {
      const int row = r0 + k;
      if (row >= rows) break;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        const int c = 8 * (hl + 32 * j);
        tx[k][j] = *(const f16x8*)(x + (int64_t)row * D + c);
        td[k][j] = *(const f16x8*)(dy + (int64_t)row * D + c);
        tr[k][j] = *(const f16x8*)(dres + (int64_t)row * D + c);
      }
    }
#pragma unroll
    for (int k = 0; k < RPH; ++k) {
      const int row = r0 + k;
      if (row >= rows) break;
#pragma unroll
      for (int j = 0; j < CH; ++j)
        *(f16x8*)(dx + (int64_t)row * D + 8 * (hl + 32 * j)) = tx[k][j] + td[k][j] + tr[k][j];
    }
    return;
  }
  bool use[RPH];
  int rws[RPH];
  float means[RPH], rstds[RPH];
#pragma unroll
  for (int k = 0; k < RPH; ++k) {
    const int row = min(r0 + k, rows - 1);
    rws[k] = row;
    use[k] = r0 + k < rows;
    means[k] = mean_in[row];
    rstds[k] = rstd_in[row];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      const int c = 8 * (hl + 32 * j);
      tx[k][j] = *(const f16x8*)(x + (int64_t)row * D + c);
      td[k][j] = *(const f16x8*)(dy + (int64_t)row * D + c);
      if (!(MODE & 8)) tr[k][j] = *(const f16x8*)(dres + (int64_t)row * D + c);
      else tr[k][j] = f16x8{};
    }
  }
#pragma unroll
  for (int k = 0; k < RPH; ++k) {
    if (use[k]) {
      const float mean = means[k], rstd = rstds[k];
      float sdg0 = 0.f, sdg1 = 0.f, sdgx0 = 0.f, sdgx1 = 0.f;
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
      f16* dxr = dx + (int64_t)rws[k] * D;
#pragma unroll
      for (int j = 0; j < CH; ++j) {
        f16x8 o;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float t = ((rstd * (float)td[k][j][e]) * gv[j * 8 + e] + b * (float)tx[k][j][e]) + c;
          o[e] = (f16)((float)tr[k][j][e] + r16(t));
        }
        if (MODE & 16) __builtin_nontemporal_store(o, (f16x8*)(dxr + 8 * (hl + 32 * j)));
        else if (!(MODE & 4) || (float)o[0] == 12345.f) *(f16x8*)(dxr + 8 * (hl + 32 * j)) = o;
      }
    }
  }
  if (MODE & 2) {
    if (accg[0] == 12345.f && accb[5] == 777.f) dg_part[blockIdx.x] = accg[1];
    return;
  }
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      red_g[hw][8 * (hl + 32 * j) + e] = accg[j * 8 + e];
      red_b[hw][8 * (hl + 32 * j) + e] = accb[j * 8 + e];
    }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += 256) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sg += red_g[k][col];
      sb += red_b[k][col];
    }
    dg_part[(int64_t)blockIdx.x * D + col] = sg;
    db_part[(int64_t)blockIdx.x * D + col] = sb;
  }
}

// Candidate: one row per half-wave, 8 waves per 16-row block (twice the waves of ln_bwd2<768, 8>), the pair of rows
// a two-row half-wave would sum added across the wave's halves (lane l + lane l ^ 32: the same fl(a + b)), so the
// LDS column reduction and the partials are those of ln_bwd2<768, 8> bit for bit; LDS stays 48 KB per block.
template <bool NT>
__global__ __launch_bounds__(512) void lnb16_kernel(const f16* __restrict__ dy, const f16* __restrict__ x,
                                                    const float* __restrict__ gamma, const float* __restrict__ mean_in,
                                                    const float* __restrict__ rstd_in, const f16* __restrict__ dres,
                                                    f16* __restrict__ dx, float* __restrict__ dg_part,
                                                    float* __restrict__ db_part, int rows) {
  constexpr int D = 768, CH = 3;
  __shared__ float red_g[8][D];
  __shared__ float red_b[8][D];
  const int hl = threadIdx.x & 31, hw = threadIdx.x >> 5, w = threadIdx.x >> 6;
  const int row = min(blockIdx.x * 16 + hw, rows - 1);
  const bool use = blockIdx.x * 16 + hw < rows;
  const float mean = mean_in[row], rstd = rstd_in[row];
  f16x8 tx[CH], td[CH], tr[CH];
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = 8 * (hl + 32 * j);
    tx[j] = *(const f16x8*)(x + (int64_t)row * D + c);
    td[j] = *(const f16x8*)(dy + (int64_t)row * D + c);
    tr[j] = *(const f16x8*)(dres + (int64_t)row * D + c);
  }
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
  if (use) {
    float sdg0 = 0.f, sdg1 = 0.f, sdgx0 = 0.f, sdgx1 = 0.f;
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float xv = (float)tx[j][e], dv = (float)td[j][e];
        const float dg = dv * gv[j * 8 + e];
        if (e < 4) {
          sdg0 += dg;
          sdgx0 += dg * xv;
        } else {
          sdg1 += dg;
          sdgx1 += dg * xv;
        }
        const float xhat = (xv - mean) * rstd;
        accg[j * 8 + e] = 0.f + dv * xhat;
        accb[j * 8 + e] = 0.f + dv;
      }
    const float sdg = half_sum(sdg0) + half_sum(sdg1);
    const float sdgx = half_sum(sdgx0) + half_sum(sdgx1);
    const float invD = 1.0f / (float)D;
    const float b = (sdg * mean - sdgx) * rstd * rstd * rstd * invD;
    const float c = -b * mean - sdg * rstd * invD;
    f16* dxr = dx + (int64_t)row * D;
#pragma unroll
    for (int j = 0; j < CH; ++j) {
      f16x8 o;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float t = ((rstd * (float)td[j][e]) * gv[j * 8 + e] + b * (float)tx[j][e]) + c;
        o[e] = (f16)((float)tr[j][e] + r16(t));
      }
      if (NT) __builtin_nontemporal_store(o, (f16x8*)(dxr + 8 * (hl + 32 * j)));
      else *(f16x8*)(dxr + 8 * (hl + 32 * j)) = o;
    }
  }
  // rows 2w and 2w + 1 of the block: the pair sum a two-row half-wave accumulates ((0 + a) + b = a + b)
#pragma unroll
  for (int i = 0; i < CH * 8; ++i) {
    accg[i] = accg[i] + __shfl_xor(accg[i], 32, 64);
    accb[i] = accb[i] + __shfl_xor(accb[i], 32, 64);
  }
  if (!(hw & 1)) {
#pragma unroll
    for (int j = 0; j < CH; ++j)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red_g[w][8 * (hl + 32 * j) + e] = accg[j * 8 + e];
        red_b[w][8 * (hl + 32 * j) + e] = accb[j * 8 + e];
      }
  }
  __syncthreads();
  for (int col = threadIdx.x; col < D; col += 512) {
    float sg = 0.f, sb = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sg += red_g[k][col];
      sb += red_b[k][col];
    }
    dg_part[(int64_t)blockIdx.x * D + col] = sg;
    db_part[(int64_t)blockIdx.x * D + col] = sb;
  }
}
}  // namespace

extern "C" int lnb_launch(int mode, const void* dy, const void* x, const float* gamma, const float* mean,
                          const float* rstd, const void* dres, void* dx, float* dg, float* db, int rows, void* stream) {
  const dim3 g((rows + 15) / 16);
  hipStream_t st = (hipStream_t)stream;
#define L(M) lnb_kernel<M><<<g, 256, 0, st>>>((const f16*)dy, (const f16*)x, gamma, mean, rstd, (const f16*)dres, \
                                             (f16*)dx, dg, db, rows)
  switch (mode) {
    case 0: L(0); break;
    case 1: L(1); break;
    case 2: L(2); break;
    case 3: L(3); break;
    case 4: L(4); break;
    case 6: L(6); break;
    case 8: L(8); break;
    case 15: L(15); break;
    case 16: L(16); break;
    case 64: L(64); break;
    case 128: lnb16_kernel<false><<<g, 512, 0, st>>>((const f16*)dy, (const f16*)x, gamma, mean, rstd, (const f16*)dres,
                                                    (f16*)dx, dg, db, rows); break;
    case 144: lnb16_kernel<true><<<g, 512, 0, st>>>((const f16*)dy, (const f16*)x, gamma, mean, rstd, (const f16*)dres,
                                                   (f16*)dx, dg, db, rows); break;
    default: return -1;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
