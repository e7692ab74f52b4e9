// Byte-moving and small kernels around the MaPLe towers (all HBM- or latency-bound):
//   * patch im2col (K1 operand; image fp32 -> fp16 cast as in trainers/maple.py:336)
//   * vision token assembly: class token, patches, +pos (fp16 add), shared ctx (clip/model.py:522-538)
//   * text prompt assembly: prefix | ctx | suffix, +pos (trainers/maple.py:152-166, :54)
//   * deep-prompt inject and its batch reduction backward (clip/model.py:320-349)
//   * fp16 transpose (dW operands), fp16 column sums (bias grads)
//   * small linears of the prompt learner (trainers/maple.py:111-131,194-215)
//   * the caption path (K19, clip/model.py:457-476, 550-561): attention pooling of the caption token
//     embeddings, and the growing vision sequence at each prompted layer (+ its backward)
#include "mf_common.h"

namespace {

// ---------------------------------------------------------------- im2col for the 16x16/16 conv
// out[b*G*G + py*G + px][c*P*P + kh*P + kw] = img[b][c][py*P+kh][px*P+kw]   (P = 16, G = R/P)
template <typename TIn>
__global__ void im2col_kernel(const TIn* __restrict__ img, f16* __restrict__ out, int B, int R, int P) {
  const int G = R / P;
  const int K = 3 * P * P;
  const int chunks_per_row = K / 8;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)B * G * G * chunks_per_row;
  if (t >= total) return;
  const int ch = t % chunks_per_row;
  const int64_t prow = t / chunks_per_row;
  const int b = prow / (G * G), pp = prow % (G * G);
  const int py = pp / G, px = pp % G;
  const int k = ch * 8;
  const int c = k / (P * P), kh = (k / P) % P, kw = k % P;
  const TIn* src = img + (((int64_t)b * 3 + c) * R + (py * P + kh)) * R + px * P + kw;
  f16x8 v;
  if constexpr (sizeof(TIn) == 4) {
    // 8 consecutive fp32 pixels: two 16-byte loads (R % 8 == 0 and P % 8 == 0 keep src 32-byte aligned)
    const f32x4 a = *(const f32x4*)src, d = *(const f32x4*)(src + 4);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      v[e] = (f16)a[e];
      v[4 + e] = (f16)d[e];
    }
  } else {
    v = *(const f16x8*)src;
  }
  *(f16x8*)(out + prow * K + k) = v;
}

// ---------------------------------------------------------------- vision token assembly
// x[b, 0]      = fp16(fp16(class_emb) + fp16(pos[0]))
// x[b, 1+p]    = fp16(patch[b, p] + fp16(pos[1+p]))
// x[b, G2+1+j] = shared_ctx[j]  (j < n_ctx)
__global__ void vision_assemble_kernel(const f16* __restrict__ patch, const float* __restrict__ cls,
                                       const float* __restrict__ pos, const f16* __restrict__ shared_ctx,
                                       f16* __restrict__ x, int B, int G2, int n_ctx, int D) {
  const int L = G2 + 1 + n_ctx;
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // over B*L*D/4
  const int64_t total = (int64_t)B * L * (D / 4);
  if (t >= total) return;
  const int d = (t % (D / 4)) * 4;
  const int64_t row = t / (D / 4);
  const int l = row % L, b = row / L;
  f16x4 o;
  if (l == 0) {
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (f16)(r16(cls[d + e]) + r16(pos[d + e]));
  } else if (l <= G2) {
    f16x4 p = *(const f16x4*)(patch + ((int64_t)b * G2 + (l - 1)) * D + d);
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = (f16)((float)p[e] + r16(pos[(int64_t)l * D + d + e]));
  } else {
    o = *(const f16x4*)(shared_ctx + (int64_t)(l - G2 - 1) * D + d);
  }
  *(f16x4*)(x + row * D + d) = o;
}

// ---------------------------------------------------------------- text prompt assembly
// x[k, l] = fp16(src[k,l] + fp16(pos[l])), src = prefix (l=0) | ctx (1..n_ctx) | suffix
__global__ void text_assemble_kernel(const f16* __restrict__ prefix, const f16* __restrict__ ctx,
                                     const f16* __restrict__ suffix, const float* __restrict__ pos,
                                     f16* __restrict__ x, int K, int L, int n_ctx, int D) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)K * L * (D / 4);
  if (t >= total) return;
  const int d = (t % (D / 4)) * 4;
  const int64_t row = t / (D / 4);
  const int l = row % L, k = row / L;
  const f16* src;
  if (l == 0)
    src = prefix + (int64_t)k * D;
  else if (l <= n_ctx)
    src = ctx + (int64_t)(l - 1) * D;
  else
    src = suffix + ((int64_t)k * (L - 1 - n_ctx) + (l - 1 - n_ctx)) * D;
  f16x4 s = *(const f16x4*)(src + d);
  f16x4 o;
#pragma unroll
  for (int e = 0; e < 4; ++e) o[e] = (f16)((float)s[e] + r16(pos[(int64_t)l * D + d + e]));
  *(f16x4*)(x + row * D + d) = o;
}

// ---------------------------------------------------------------- deep prompt inject
// x[n*L + row0 + r, :] = fp16(prompt[r, :])  (prompt fp32, the `.half()` at clip/model.py:327,344)
__global__ void inject_kernel(f16* __restrict__ x, const float* __restrict__ prompt, int N, int L, int row0,
                              int nrows, int D) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = N * nrows * D;
  if (t >= total) return;
  const int d = t % D;
  const int r = (t / D) % nrows;
  const int n = t / (D * nrows);
  x[((int64_t)n * L + row0 + r) * D + d] = (f16)prompt[r * D + d];
}

// out[r, d] (=|+=) sum_n dx[n*L + row0 + r, d]  (fp32 accumulation in a fixed order), then the
// injected rows of dx are zeroed (the previous layer's outputs there were discarded).
// out_f16: round once to fp16 (fp16 source tensors, e.g. ctx / shared_ctx); else fp32.
// grid (ceil(D/256), nrows), 1024 threads: lane -> 4 consecutive columns, 16 wave groups split the
// batch (n = g, g+16, ...), partials combined through LDS in group order.
__global__ __launch_bounds__(1024) void inject_bwd_kernel(f16* __restrict__ dx, int N, int L, int row0, int nrows,
                                                          int D, void* out, int out_f16, int accumulate,
                                                          int zero_rows) {
  __shared__ f32x4 red[16][64];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int r = blockIdx.y;
  const int d = blockIdx.x * 256 + lane * 4;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (d < D) {
    for (int n = g; n < N; n += 16) {
      f16x4* p = (f16x4*)(dx + ((int64_t)n * L + row0 + r) * D + d);
      const f16x4 v = *p;
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += (float)v[e];
      if (zero_rows) *p = (f16x4){(f16)0.f, (f16)0.f, (f16)0.f, (f16)0.f};
    }
  }
  red[g][lane] = s;
  __syncthreads();
  if (g == 0 && d < D) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int k = 1; k < 16; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] += red[k][lane][e];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int i = r * D + d + e;
      if (out_f16) {
        f16* o = (f16*)out + i;
        *o = accumulate ? (f16)((float)*o + r16(t[e])) : (f16)t[e];
      } else {
        float* o = (float*)out + i;
        *o = accumulate ? *o + t[e] : t[e];
      }
    }
  }
}

// ---------------------------------------------------------------- caption path (K19)
// Growing sequence at a prompted vision layer with captions (clip/model.py:320-333 fed by :558-559):
// dst[n, r] = src[n, r]                      r <  Lp - n_ctx   (all but the previous prompt rows)
//           = cap[r - (Lp - n_ctx)]           next ncap rows    (the projected captions, shared by all n)
//           = fp16(prompt[r - (L - n_ctx)])   last n_ctx rows   (the layer's deep prompt, .half())
// L = Lp + ncap.  8 fp16 per thread.
__global__ void seq_grow_kernel(const f16* __restrict__ src, f16* __restrict__ dst, const f16* __restrict__ cap,
                                const float* __restrict__ prompt, int N, int Lp, int L, int n_ctx, int D) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)N * L * (D / 8);
  if (t >= total) return;
  const int d = (int)(t % (D / 8)) * 8;
  const int64_t row = t / (D / 8);
  const int r = (int)(row % L), n = (int)(row / L);
  const int keep = Lp - n_ctx;
  f16x8 v;
  if (r < keep) {
    v = *(const f16x8*)(src + ((int64_t)n * Lp + r) * D + d);
  } else if (r < L - n_ctx) {
    v = *(const f16x8*)(cap + (int64_t)(r - keep) * D + d);
  } else {
    const float* p = prompt + (int64_t)(r - (L - n_ctx)) * D + d;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = (f16)p[e];
  }
  *(f16x8*)(dst + row * D + d) = v;
}

// its backward into the previous layer's output: dsrc[n, r] = ddst[n, r] for r < Lp - n_ctx, 0 for the
// previous prompt rows the layer dropped (the caption rows' and the prompt rows' gradients go elsewhere)
__global__ void seq_grow_bwd_kernel(const f16* __restrict__ ddst, f16* __restrict__ dsrc, int N, int Lp, int L,
                                    int n_ctx, int D) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t total = (int64_t)N * Lp * (D / 8);
  if (t >= total) return;
  const int d = (int)(t % (D / 8)) * 8;
  const int64_t row = t / (D / 8);
  const int r = (int)(row % Lp), n = (int)(row / Lp);
  f16x8 v = {};
  if (r < Lp - n_ctx) v = *(const f16x8*)(ddst + ((int64_t)n * L + r) * D + d);
  *(f16x8*)(dsrc + row * D + d) = v;
}

// AttentionPooling over one caption per block (clip/model.py:464-476), from the token ids:
//   emb[t] = fp16(token_embedding[tok[t]])                      (.type(fp16), trainers/maple.py:316)
//   s[t]   = fp16(emb[t] . w)                                   (torch.matmul, fp32 accumulate)
//   p      = fp16(softmax(s))                                   (over the T <= 128 tokens, fp32 math)
//   pooled = fp16(sum_t fp16(emb[t] * p[t]))                    (fp32 accumulate, tokens in order)
// one wave per token for the scores, one thread per column for the pooled sum.  An id outside [0, vocab)
// reads no table row: its score is NaN, so the caption's pooled row is NaN and the step's loss check fails
// loudly (the host range-checks ids before the upload; this guards direct device callers).
__global__ __launch_bounds__(256) void caption_pool_kernel(const int* __restrict__ tok, int T,
                                                           const float* __restrict__ table, int vocab,
                                                           const f16* __restrict__ w, int D, f16* __restrict__ pooled) {
  __shared__ float s_score[128];
  __shared__ float s_p[128];
  const int b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int* tb = tok + (int64_t)b * T;
  for (int t = wv; t < T; t += 4) {
    const int id = tb[t];
    if (id < 0 || id >= vocab) {
      if (lane == 0) s_score[t] = NAN;
      continue;
    }
    const float* e = table + (int64_t)id * D;
    float s = 0.f;
    for (int d = lane; d < D; d += 64) s += (float)(f16)e[d] * (float)w[d];
    s = wave_sum(s);
    if (lane == 0) s_score[t] = r16(s);
  }
  __syncthreads();
  if (wv == 0) {
    float m = -INFINITY;
    for (int t = lane; t < T; t += 64) m = fmaxf(m, s_score[t]);
    m = wave_max(m);
    float z = 0.f;
    for (int t = lane; t < T; t += 64) z += expf(s_score[t] - m);
    z = wave_sum(z);
    for (int t = lane; t < T; t += 64) s_p[t] = r16(expf(s_score[t] - m) / z);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float acc = 0.f;
    for (int t = 0; t < T; ++t) {
      const int id = tb[t];
      const float e = (id >= 0 && id < vocab) ? (float)(f16)table[(int64_t)id * D + d] : 0.f;
      acc += r16(e * s_p[t]);
    }
    pooled[(int64_t)b * D + d] = (f16)acc;
  }
}

// ---------------------------------------------------------------- transpose [R,C] -> [C,R]
// 64 x 64 tiles, 256 threads: 16-byte loads (8 fp16 of a row) into a padded LDS tile, 16-byte stores
// (8 fp16 of an output row = 8 input rows of one column).  Ragged edges fall back to element access.
__global__ __launch_bounds__(256) void transpose_kernel(const f16* __restrict__ in, int64_t ld_in,
                                                       f16* __restrict__ out, int64_t ld_out, int R, int C) {
  __shared__ f16 tile[64][72];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  const int t = threadIdx.x;
  const bool full = r0 + 64 <= R && c0 + 64 <= C && (ld_in % 8) == 0 && (ld_out % 8) == 0 &&
                    ((uintptr_t)in % 16) == 0 && ((uintptr_t)out % 16) == 0;
  if (full) {
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int r = t / 8 + 32 * k, c8 = (t % 8) * 8;
      *(f16x8*)&tile[r][c8] = *(const f16x8*)(in + (int64_t)(r0 + r) * ld_in + c0 + c8);
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const int c = t / 8 + 32 * k, r8 = (t % 8) * 8;
      f16x8 v;
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = tile[r8 + e][c];
      *(f16x8*)(out + (int64_t)(c0 + c) * ld_out + r0 + r8) = v;
    }
    return;
  }
  const int tx = t & 63, ty = t >> 6;
  for (int i = ty; i < 64; i += 4) {
    const int r = r0 + i, c = c0 + tx;
    tile[i][tx] = (r < R && c < C) ? in[(int64_t)r * ld_in + c] : (f16)0.f;
  }
  __syncthreads();
  for (int i = ty; i < 64; i += 4) {
    const int c = c0 + i, r = r0 + tx;
    if (c < C && r < R) out[(int64_t)c * ld_out + r] = tile[tx][i];
  }
}

// ---------------------------------------------------------------- column sums (bias grads)
// part[chunk][c] = sum of rows [64*chunk, 64*chunk+64) of column c: a block of 256 threads covers
// 256 columns (4 per lane, 8-byte loads) x 64 rows (16 per wave); then col_reduce_kernel.
constexpr int CS_ROWS = 64;
__global__ __launch_bounds__(256) void colsum_part_kernel(const f16* __restrict__ in, int64_t ld, int R, int C,
                                                          float* __restrict__ part) {
  __shared__ f32x4 red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 256 + lane * 4;
  const int r0 = blockIdx.y * CS_ROWS + w * 16;
  f32x4 s = {0.f, 0.f, 0.f, 0.f};
  if (c < C) {
#pragma unroll 4
    for (int r = r0; r < min(R, r0 + 16); ++r) {
      f16x4 v = *(const f16x4*)(in + (int64_t)r * ld + c);
#pragma unroll
      for (int e = 0; e < 4; ++e) s[e] += (float)v[e];
    }
  }
  red[w][lane] = s;
  __syncthreads();
  if (w == 0 && c < C) {
    f32x4 t = red[0][lane];
#pragma unroll
    for (int k = 1; k < 4; ++k)
#pragma unroll
      for (int e = 0; e < 4; ++e) t[e] += red[k][lane][e];
    *(f32x4*)(part + (int64_t)blockIdx.y * C + c) = t;
  }
}

// ---------------------------------------------------------------- small linears (M rows <= 16)
// Y[m,o] = X[m,:] . W[o,:] + b[o]  (T = float: fp32 Linear, T = f16: fp16 Linear rounded once)
template <typename T>
__global__ void small_linear_fwd_kernel(const T* __restrict__ X, const T* __restrict__ W, const T* __restrict__ b,
                                        T* __restrict__ Y, int M, int I, int O) {
  const int wave = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wave >= M * O) return;
  const int m = wave / O, o = wave % O;
  float s = 0.f;
  for (int i = lane; i < I; i += 64) s += (float)X[(int64_t)m * I + i] * (float)W[(int64_t)o * I + i];
  s = wave_sum(s);
  if (lane == 0) Y[(int64_t)m * O + o] = (T)(s + (b ? (float)b[o] : 0.f));
}
// dX[m,i] (=|+=) sum_o dY[m,o] W[o,i]   ; fp16 accumulate rounds the new term once then adds.
// grid (I/64, M), 1024 threads: lane -> column i, 16 wave groups split the o range (fixed order
// LDS reduction), so the O-long dot product is 16-way parallel instead of one serial chain.
template <typename T>
__global__ __launch_bounds__(1024) void small_linear_bwd_dx_kernel(const T* __restrict__ dY,
                                                                   const T* __restrict__ W, T* __restrict__ dX,
                                                                   int M, int I, int O, int accumulate) {
  __shared__ float red[16][65];
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane, m = blockIdx.y;
  float s0 = 0.f, s1 = 0.f;
  if (i < I) {
    int o = g;
    for (; o + 16 < O; o += 32) {
      s0 += (float)dY[(int64_t)m * O + o] * (float)W[(int64_t)o * I + i];
      s1 += (float)dY[(int64_t)m * O + o + 16] * (float)W[(int64_t)(o + 16) * I + i];
    }
    for (; o < O; o += 16) s0 += (float)dY[(int64_t)m * O + o] * (float)W[(int64_t)o * I + i];
  }
  red[g][lane] = s0 + s1;
  __syncthreads();
  if (g == 0 && i < I) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][lane];
    const int64_t t = (int64_t)m * I + i;
    if (accumulate)
      dX[t] = (T)((float)dX[t] + (float)(T)s);
    else
      dX[t] = (T)s;
  }
}
// dW[o,i] = sum_m dY[m,o] X[m,i] ; db[o] = sum_m dY[m,o]
template <typename T>
__global__ void small_linear_bwd_dw_kernel(const T* __restrict__ dY, const T* __restrict__ X, T* __restrict__ dW,
                                           T* __restrict__ db, int M, int I, int O) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= O * I) return;
  const int o = t / I, i = t % I;
  float s = 0.f;
  for (int m = 0; m < M; ++m) s += (float)dY[(int64_t)m * O + o] * (float)X[(int64_t)m * I + i];
  dW[t] = (T)s;
  if (i == 0 && db) {
    float sb = 0.f;
    for (int m = 0; m < M; ++m) sb += (float)dY[(int64_t)m * O + o];
    db[o] = (T)sb;
  }
}

// ---------------------------------------------------------------- batched small linears
// Every Linear of the prompt learner (proj_lang_to_vis on ctx, the J-1 compound prompt projections)
// in ONE launch per direction, driven by a device descriptor table: they are independent of each
// other in both directions (distinct outputs, distinct gradient targets), and each is far too small
// to fill the chip alone (<= 2 x 768 outputs), so their launch latencies were the cost.
struct LinDesc {
  const void* X;   // [M, I]
  const void* W;   // [O, I]
  const void* b;   // [O] or null
  void* Y;         // [M, O]
  const void* dY;  // [M, O]
  void* dX;        // [M, I] or null (accumulated when acc_dx)
  void* dW;        // [O, I] or null
  void* db;        // [O] or null
  int M, I, O, is16, acc_dx, pad;
};

template <typename T>
MF_DEV float ldv(const void* p, int64_t i) { return (float)((const T*)p)[i]; }

// grid (ceil(maxMO / 4), n): wave w of block x computes output (m, o) = 4x + w of descriptor y
__global__ __launch_bounds__(256) void lin_fwd_batch_kernel(const LinDesc* __restrict__ descs) {
  const LinDesc d = descs[blockIdx.y];
  const int idx = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (idx >= d.M * d.O) return;
  const int m = idx / d.O, o = idx % d.O;
  float s = 0.f;
  if (d.is16) {
    for (int i = lane; i < d.I; i += 64) s += ldv<f16>(d.X, (int64_t)m * d.I + i) * ldv<f16>(d.W, (int64_t)o * d.I + i);
  } else {
    for (int i = lane; i < d.I; i += 64) s += ldv<float>(d.X, (int64_t)m * d.I + i) * ldv<float>(d.W, (int64_t)o * d.I + i);
  }
  s = wave_sum(s);
  if (lane == 0) {
    if (d.is16)
      ((f16*)d.Y)[(int64_t)m * d.O + o] = (f16)(s + (d.b ? ldv<f16>(d.b, o) : 0.f));
    else
      ((float*)d.Y)[(int64_t)m * d.O + o] = s + (d.b ? ldv<float>(d.b, o) : 0.f);
  }
}

// dX[m,i] (=|+=) sum_o dY[m,o] W[o,i]: grid (ceil(maxI/64), maxM, n), 1024 threads, 16 wave groups
// split the o range (fixed-order LDS reduction: deterministic), as small_linear_bwd_dx_kernel
__global__ __launch_bounds__(1024) void lin_bwd_dx_batch_kernel(const LinDesc* __restrict__ descs) {
  __shared__ float red[16][65];
  const LinDesc d = descs[blockIdx.z];
  if (!d.dX || (int)blockIdx.y >= d.M || (int)blockIdx.x * 64 >= d.I) return;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane, m = blockIdx.y;
  float s0 = 0.f, s1 = 0.f;
  if (i < d.I) {
    int o = g;
    if (d.is16) {
      for (; o + 16 < d.O; o += 32) {
        s0 += ldv<f16>(d.dY, (int64_t)m * d.O + o) * ldv<f16>(d.W, (int64_t)o * d.I + i);
        s1 += ldv<f16>(d.dY, (int64_t)m * d.O + o + 16) * ldv<f16>(d.W, (int64_t)(o + 16) * d.I + i);
      }
      for (; o < d.O; o += 16) s0 += ldv<f16>(d.dY, (int64_t)m * d.O + o) * ldv<f16>(d.W, (int64_t)o * d.I + i);
    } else {
      for (; o + 16 < d.O; o += 32) {
        s0 += ldv<float>(d.dY, (int64_t)m * d.O + o) * ldv<float>(d.W, (int64_t)o * d.I + i);
        s1 += ldv<float>(d.dY, (int64_t)m * d.O + o + 16) * ldv<float>(d.W, (int64_t)(o + 16) * d.I + i);
      }
      for (; o < d.O; o += 16) s0 += ldv<float>(d.dY, (int64_t)m * d.O + o) * ldv<float>(d.W, (int64_t)o * d.I + i);
    }
  }
  red[g][lane] = s0 + s1;
  __syncthreads();
  if (g == 0 && i < d.I) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][lane];
    const int64_t t = (int64_t)m * d.I + i;
    if (d.is16) {
      f16* dx = (f16*)d.dX;
      dx[t] = d.acc_dx ? (f16)((float)dx[t] + (float)(f16)s) : (f16)s;
    } else {
      float* dx = (float*)d.dX;
      dx[t] = d.acc_dx ? dx[t] + s : s;
    }
  }
}

// dW[o,i] = sum_m dY[m,o] X[m,i];  db[o] = sum_m dY[m,o]:  grid (ceil(maxOI/256), n)
__global__ __launch_bounds__(256) void lin_bwd_dw_batch_kernel(const LinDesc* __restrict__ descs) {
  const LinDesc d = descs[blockIdx.y];
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (!d.dW || t >= d.O * d.I) return;
  const int o = t / d.I, i = t % d.I;
  float s = 0.f, sb = 0.f;
  if (d.is16) {
    for (int m = 0; m < d.M; ++m) {
      const float gy = ldv<f16>(d.dY, (int64_t)m * d.O + o);
      s += gy * ldv<f16>(d.X, (int64_t)m * d.I + i);
      sb += gy;
    }
    ((f16*)d.dW)[t] = (f16)s;
    if (i == 0 && d.db) ((f16*)d.db)[o] = (f16)sb;
  } else {
    for (int m = 0; m < d.M; ++m) {
      const float gy = ldv<float>(d.dY, (int64_t)m * d.O + o);
      s += gy * ldv<float>(d.X, (int64_t)m * d.I + i);
      sb += gy;
    }
    ((float*)d.dW)[t] = s;
    if (i == 0 && d.db) ((float*)d.db)[o] = sb;
  }
}

// ---------------------------------------------------------------- casts
__global__ void cast_f16_to_f32_kernel(const f16* __restrict__ in, float* __restrict__ out, int64_t n) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t < n) out[t] = (float)in[t];
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

extern "C" int mf_im2col_patch(const void* img, int img_is_f32, void* out, int B, int R, int P, void* stream) {
  if (B <= 0) return 0;
  if (R % P || (3 * P * P) % 8 || P % 8) return mf_set_error("mf_im2col_patch: bad geometry", -1);
  if ((uintptr_t)img % 16 || (uintptr_t)out % 16) return mf_set_error("mf_im2col_patch: 16-byte aligned buffers required", -1);
  const int G = R / P;
  const int64_t total = (int64_t)B * G * G * (3 * P * P / 8);
  hipStream_t st = (hipStream_t)stream;
  if (img_is_f32)
    im2col_kernel<float><<<nblk(total), 256, 0, st>>>((const float*)img, (f16*)out, B, R, P);
  else
    im2col_kernel<f16><<<nblk(total), 256, 0, st>>>((const f16*)img, (f16*)out, B, R, P);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_vision_assemble(const void* patch, const float* cls, const float* pos, const void* shared_ctx,
                                  void* x, int B, int G2, int n_ctx, int D, void* stream) {
  if (B <= 0) return 0;
  if (D % 4) return mf_set_error("mf_vision_assemble: D % 4", -1);
  const int64_t total = (int64_t)B * (G2 + 1 + n_ctx) * (D / 4);
  vision_assemble_kernel<<<nblk(total), 256, 0, (hipStream_t)stream>>>(
      (const f16*)patch, cls, pos, (const f16*)shared_ctx, (f16*)x, B, G2, n_ctx, D);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_text_assemble(const void* prefix, const void* ctx, const void* suffix, const float* pos, void* x,
                                int K, int L, int n_ctx, int D, void* stream) {
  if (K <= 0) return 0;
  if (D % 4) return mf_set_error("mf_text_assemble: D % 4", -1);
  const int64_t total = (int64_t)K * L * (D / 4);
  text_assemble_kernel<<<nblk(total), 256, 0, (hipStream_t)stream>>>(
      (const f16*)prefix, (const f16*)ctx, (const f16*)suffix, pos, (f16*)x, K, L, n_ctx, D);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_prompt_inject_fwd(void* x, const float* prompt, int N, int L, int row0, int nrows, int D,
                                    void* stream) {
  if (N <= 0) return 0;
  if (row0 < 0 || row0 + nrows > L) return mf_set_error("mf_prompt_inject_fwd: rows out of range", -1);
  inject_kernel<<<nblk((int64_t)N * nrows * D), 256, 0, (hipStream_t)stream>>>((f16*)x, prompt, N, L, row0, nrows, D);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_prompt_inject_bwd(void* dx, int N, int L, int row0, int nrows, int D, void* out, int out_f16,
                                    int accumulate, int zero_rows, void* stream) {
  if (row0 < 0 || row0 + nrows > L) return mf_set_error("mf_prompt_inject_bwd: rows out of range", -1);
  if (D % 4) return mf_set_error("mf_prompt_inject_bwd: D % 4", -1);
  inject_bwd_kernel<<<dim3((D + 255) / 256, nrows), 1024, 0, (hipStream_t)stream>>>((f16*)dx, N, L, row0, nrows, D,
                                                                                    out, out_f16, accumulate,
                                                                                    zero_rows);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_seq_grow(const void* src, void* dst, const void* cap, const float* prompt, int N, int Lp, int ncap,
                           int n_ctx, int D, void* stream) {
  if (N <= 0) return 0;
  if (D % 8 || Lp < n_ctx || ncap < 0 || n_ctx < 0) return mf_set_error("mf_seq_grow: bad shape", -1);
  const int L = Lp + ncap;
  const int64_t total = (int64_t)N * L * (D / 8);
  seq_grow_kernel<<<nblk(total), 256, 0, (hipStream_t)stream>>>((const f16*)src, (f16*)dst, (const f16*)cap, prompt,
                                                               N, Lp, L, n_ctx, D);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_seq_grow_bwd(const void* ddst, void* dsrc, int N, int Lp, int ncap, int n_ctx, int D, void* stream) {
  if (N <= 0) return 0;
  if (D % 8 || Lp < n_ctx || ncap < 0) return mf_set_error("mf_seq_grow_bwd: bad shape", -1);
  const int64_t total = (int64_t)N * Lp * (D / 8);
  seq_grow_bwd_kernel<<<nblk(total), 256, 0, (hipStream_t)stream>>>((const f16*)ddst, (f16*)dsrc, N, Lp, Lp + ncap,
                                                                   n_ctx, D);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_caption_pool(const int* tokens, int B, int T, const float* table, int vocab, const void* w, int D,
                               void* pooled, void* stream) {
  if (B <= 0) return 0;
  if (T <= 0 || T > 128) return mf_set_error("mf_caption_pool: 0 < T <= 128 tokens", -1);
  if (vocab <= 0) return mf_set_error("mf_caption_pool: vocab must be positive", -1);
  caption_pool_kernel<<<B, 256, 0, (hipStream_t)stream>>>(tokens, T, table, vocab, (const f16*)w, D, (f16*)pooled);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_transpose_f16(const void* in, int64_t ld_in, void* out, int64_t ld_out, int R, int C,
                                void* stream) {
  if (R <= 0 || C <= 0) return 0;
  dim3 grid((C + 63) / 64, (R + 63) / 64);
  transpose_kernel<<<grid, 256, 0, (hipStream_t)stream>>>((const f16*)in, ld_in, (f16*)out, ld_out, R, C);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_colsum_blocks(int R) { return (R + CS_ROWS - 1) / CS_ROWS; }

extern "C" int mf_colsum_f16(const void* in, int64_t ld, int R, int C, void* out, int out_f16, float* workspace,
                             void* stream) {
  if (R <= 0 || C <= 0) return 0;
  const int nb = mf_colsum_blocks(R);
  hipStream_t st = (hipStream_t)stream;
  if (C % 4 || ld % 4) return mf_set_error("mf_colsum_f16: C and ld must be multiples of 4", -1);
  dim3 grid((C + 255) / 256, nb);
  colsum_part_kernel<<<grid, 256, 0, st>>>((const f16*)in, ld, R, C, workspace);
  MF_CHECK_LAUNCH();
  if (out_f16)
    col_reduce_kernel<true><<<dim3((C + 63) / 64, 1), 1024, 0, st>>>(workspace, workspace, nb, C, C, out, out, 0);
  else
    col_reduce_kernel<false><<<dim3((C + 63) / 64, 1), 1024, 0, st>>>(workspace, workspace, nb, C, C, out, out, 0);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_small_linear_fwd(const void* X, const void* W, const void* b, void* Y, int M, int I, int O,
                                   int is_f16, void* stream) {
  if (M <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const int64_t threads = (int64_t)M * O * 64;
  if (is_f16)
    small_linear_fwd_kernel<f16><<<nblk(threads), 256, 0, st>>>((const f16*)X, (const f16*)W, (const f16*)b, (f16*)Y,
                                                               M, I, O);
  else
    small_linear_fwd_kernel<float><<<nblk(threads), 256, 0, st>>>((const float*)X, (const float*)W,
                                                                  (const float*)b, (float*)Y, M, I, O);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_small_linear_bwd(const void* dY, const void* X, const void* W, void* dX, void* dW, void* db, int M,
                                   int I, int O, int is_f16, int accumulate_dx, void* stream) {
  if (M <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  if (is_f16) {
    if (dX)
      small_linear_bwd_dx_kernel<f16><<<dim3((I + 63) / 64, M), 1024, 0, st>>>((const f16*)dY, (const f16*)W,
                                                                                (f16*)dX, M, I, O, accumulate_dx);
    if (dW)
      small_linear_bwd_dw_kernel<f16><<<nblk((int64_t)O * I), 256, 0, st>>>((const f16*)dY, (const f16*)X, (f16*)dW,
                                                                            (f16*)db, M, I, O);
  } else {
    if (dX)
      small_linear_bwd_dx_kernel<float><<<dim3((I + 63) / 64, M), 1024, 0, st>>>(
          (const float*)dY, (const float*)W, (float*)dX, M, I, O, accumulate_dx);
    if (dW)
      small_linear_bwd_dw_kernel<float><<<nblk((int64_t)O * I), 256, 0, st>>>((const float*)dY, (const float*)X,
                                                                              (float*)dW, (float*)db, M, I, O);
  }
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_cast_f16_f32(const void* in, float* out, int64_t n, void* stream) {
  if (n <= 0) return 0;
  cast_f16_to_f32_kernel<<<nblk(n), 256, 0, (hipStream_t)stream>>>((const f16*)in, out, n);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_small_linear_desc_bytes(void) { return (int)sizeof(LinDesc); }

extern "C" int mf_small_linear_fwd_batch(const void* descs, int n, int max_mo, void* stream) {
  if (n <= 0 || max_mo <= 0) return 0;
  lin_fwd_batch_kernel<<<dim3((max_mo + 3) / 4, n), 256, 0, (hipStream_t)stream>>>((const LinDesc*)descs);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_small_linear_bwd_batch(const void* descs, int n, int max_m, int max_i, int max_oi, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  lin_bwd_dx_batch_kernel<<<dim3((max_i + 63) / 64, max_m, n), 1024, 0, st>>>((const LinDesc*)descs);
  MF_CHECK_LAUNCH();
  lin_bwd_dw_batch_kernel<<<dim3((max_oi + 255) / 256, n), 256, 0, st>>>((const LinDesc*)descs);
  MF_CHECK_LAUNCH();
  return 0;
}

namespace {
__global__ void seq_scatter_kernel(const f16* __restrict__ src, int64_t ld_src, f16* __restrict__ dst, int64_t ld_dst,
                                   int L_live, int L_full, int C8, int64_t total) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const int64_t row = i / C8;
  const int c = (int)(i % C8) * 8;
  const int64_t n = row / L_live, t = row % L_live;
  *(f16x8*)(dst + (n * L_full + t) * ld_dst + c) = *(const f16x8*)(src + row * ld_src + c);
}
}  // namespace

// Rows of N compact L_live-row sequences into the first L_live rows of N L_full-row sequences (dst row
// n * L_full + t = src row n * L_live + t; dst's other rows untouched).  The EOT-truncated text tower's operands
// of its block-11 weight gradients, laid out as the full-length tower's (whose extra rows are zero).
extern "C" int mf_seq_scatter(const void* src, int64_t ld_src, void* dst, int64_t ld_dst, int N, int L_live,
                              int L_full, int C, void* stream) {
  if (N <= 0 || C <= 0) return 0;
  if (L_live <= 0 || L_live > L_full || C % 8 || ld_src % 8 || ld_dst % 8 || ld_src < C || ld_dst < C ||
      (uintptr_t)src % 16 || (uintptr_t)dst % 16)
    return mf_set_error("mf_seq_scatter: bad shape or alignment", -1);
  const int64_t total = (int64_t)N * L_live * (C / 8);
  seq_scatter_kernel<<<nblk(total), 256, 0, (hipStream_t)stream>>>((const f16*)src, ld_src, (f16*)dst, ld_dst, L_live,
                                                                  L_full, C / 8, total);
  MF_CHECK_LAUNCH();
  return 0;
}
