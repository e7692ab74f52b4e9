// Cosine-logit head and MaPLe loss (trainers/maple.py:325,340-378):
//   img_n = F.normalize(img, eps=1e-8), txt_n = F.normalize(txt, eps=1e-8)  (fp16: x / fp16(||x||))
//   logits = fp16(min(exp(logit_scale),100) * fp16(img_n @ txt_n^T))
//   loss   = CE(logits, y) + 0.5 * (1 - mean_b cos(img_n[b], txt_n[y_b]))
// or, for soft (float) labels q [B,K] (trainers/maple.py:356-360),
//   loss   = KL(q.clamp(1e-8) || softmax) (batchmean, fp32) + 0.5 * (1 - mean_b cos(img_n[b], (q @ txt_n)[b]))
// and the analytic backward to d img / d txt (fp32 math, fp16 outputs at the tensor boundaries
// the reference materialises).  Small: B <= 64 rows, K <= 1000 classes, width 512.
#include "mf_common.h"

namespace {

// one wave per row: y = fp16(x / fp16(norm)); norm16 saved
__global__ void normalize_rows_kernel(const f16* __restrict__ x, f16* __restrict__ y, float* __restrict__ norm,
                                      int rows, int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const f16* xr = x + (int64_t)row * D;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) {
    float v = (float)xr[d];
    s += v * v;
  }
  s = wave_sum(s);
  float n16 = r16(sqrtf(s));
  n16 = fmaxf(n16, 1e-8f);
  for (int d = lane; d < D; d += 64) y[(int64_t)row * D + d] = (f16)((float)xr[d] / n16);
  if (lane == 0) norm[row] = n16;
}

// one wave per (b, k): mm = fp16(dot), logits = fp16(scale * mm)
__global__ void logits_kernel(const f16* __restrict__ img_n, const f16* __restrict__ txt_n, int B, int K, int D,
                              const float* __restrict__ logit_scale, f16* __restrict__ mm, f16* __restrict__ logits) {
  const int64_t w = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (w >= (int64_t)B * K) return;
  const int b = w / K, k = w % K;
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += (float)img_n[(int64_t)b * D + d] * (float)txt_n[(int64_t)k * D + d];
  s = wave_sum(s);
  if (lane == 0) {
    const float sc = fminf(expf(logit_scale[0]), 100.f);
    const float m16 = r16(s);
    mm[w] = (f16)m16;
    logits[w] = (f16)mul32(sc, m16);  // fp32 product, then fp16 (mf_common.h mul32)
  }
}

// Single block of 1024 threads (16 waves); wave w handles rows b = w, w+16, ...
// out: loss_out[0] = total (fp16 value as fp32), [1] = CE, [2] = alignment, [3] = nonfinite flag
// dmm[b,k] = fp16(fp16((softmax - onehot)/B) * scale);  cosg[b] = d cos[b] = fp16(-0.5/B)
// cos needs u = fp16(img_n/||img_n||16), v = fp16(t/||t||16) (cosine_similarity normalises again)
__global__ void loss_kernel(const f16* __restrict__ logits, const f16* __restrict__ img_n,
                            const f16* __restrict__ txt_n, const int64_t* __restrict__ label, int B, int K, int D,
                            const float* __restrict__ logit_scale, f16* __restrict__ dmm,
                            float* __restrict__ cos_out, float* __restrict__ loss_out) {
  __shared__ float s_ce[64], s_cos[64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const float sc = fminf(expf(logit_scale[0]), 100.f);
  for (int b = w; b < B; b += nw) {
    const f16* lr = logits + (int64_t)b * K;
    // a label outside [0, K) (the reference asserts, trainers/maple.py:352-353) is not indexed: the row's
    // loss becomes NaN, so the step is flagged non-finite and its update skipped
    const int y_raw = (int)label[b];
    const bool y_bad = y_raw < 0 || y_raw >= K;
    const int y = y_bad ? 0 : y_raw;
    float mx = -INFINITY;
    for (int k = lane; k < K; k += 64) mx = fmaxf(mx, (float)lr[k]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += expf((float)lr[k] - mx);
    se = wave_sum(se);
    const float lse = logf(se);
    const float logp_y = r16((float)lr[y] - mx - lse);  // log_softmax output is fp16
    // d logits = fp16((softmax - onehot) / B), then * scale -> dmm (fp16)
    for (int k = lane; k < K; k += 64) {
      const float logp = r16((float)lr[k] - mx - lse);
      const float g_nll = (k == y) ? r16(-1.0f / (float)B) : 0.f;
      // log_softmax backward: g - exp(out) * sum(g)
      const float dl = r16(g_nll - expf(logp) * r16(-1.0f / (float)B));
      dmm[(int64_t)b * K + k] = (f16)mul32(dl, sc);
    }
    // cosine similarity of img_n[b] and txt_n[y]
    float su = 0.f, sv = 0.f;
    for (int d = lane; d < D; d += 64) {
      float a = (float)img_n[(int64_t)b * D + d], t = (float)txt_n[(int64_t)y * D + d];
      su += a * a;
      sv += t * t;
    }
    const float nu = fmaxf(r16(sqrtf(wave_sum(su))), 1e-8f), nv = fmaxf(r16(sqrtf(wave_sum(sv))), 1e-8f);
    float c = 0.f;
    for (int d = lane; d < D; d += 64) {
      float a = r16((float)img_n[(int64_t)b * D + d] / nu), t = r16((float)txt_n[(int64_t)y * D + d] / nv);
      c += r16(a * t);
    }
    c = r16(wave_sum(c));
    if (lane == 0) {
      s_ce[b] = y_bad ? __builtin_nanf("") : -logp_y;
      s_cos[b] = c;
      cos_out[2 * b] = nu;
      cos_out[2 * b + 1] = nv;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float ce = 0.f, cs = 0.f;
    for (int b = 0; b < B; ++b) {
      ce += s_ce[b];
      cs += s_cos[b];
    }
    ce = r16(ce / (float)B);
    const float align = r16(1.f - r16(cs / (float)B));
    const float total = r16(ce + r16(0.5f * align));
    loss_out[0] = total;
    loss_out[1] = ce;
    loss_out[2] = align;
    loss_out[3] = isfinite(total) ? 0.f : 1.f;
  }
}

// d img_n[b,:] = fp16( fp16(sum_k dmm[b,k] txt_n[k,:]) + cos-path ) ; block per row b
// cos path (fp32): g_u = dcos*v, d img_n += g_u/nu - img_n*(g_u . img_n)/nu^3 with dcos = fp16(-0.5/B)
// soft_rows != null: the cosine target of row b is soft_rows[b,:] ((q @ txt_n)[b]) instead of txt_n[y_b]
// One wave per (row b, 64-column chunk): grid (B, ceil(D/64)).  The K-long sum of a column runs in k order
// in one lane (as before), with its loads issued 16 ahead of the FMA chain; g_u . img_n keeps the reduction
// order of the former 256-thread block (virtual thread t = lane + 64 w sums d = t, t + 256, ..; the four
// virtual waves' wave_sums added in order), so the result is bit-identical to the one-block-per-row form
// (which ran 32 blocks and took 342 us at K = 1 000).
__global__ __launch_bounds__(64) void dimg_kernel(const f16* __restrict__ dmm, const f16* __restrict__ img_n,
                                                  const f16* __restrict__ txt_n, const int64_t* __restrict__ label,
                                                  const f16* __restrict__ soft_rows,
                                                  const float* __restrict__ cos_norms, int B, int K, int D,
                                                  f16* __restrict__ dimg_n) {
  const int b = blockIdx.x, lane = threadIdx.x;
  const int y_raw = soft_rows ? 0 : (int)label[b];
  const f16* trow = soft_rows ? soft_rows + (int64_t)b * D : txt_n + (int64_t)((y_raw < 0 || y_raw >= K) ? 0 : y_raw) * D;
  const float dcos = r16(-0.5f / (float)B);
  const float nu = cos_norms[2 * b], nv = cos_norms[2 * b + 1];
  const f16* irow = img_n + (int64_t)b * D;
  // g_u . img_n
  float dotp = 0.f;
#pragma unroll
  for (int w = 0; w < 4; ++w) {
    float part = 0.f;
    for (int d = lane + 64 * w; d < D; d += 256) {
      float v = r16((float)trow[d] / nv);
      part += dcos * v * (float)irow[d];
    }
    dotp += wave_sum(part);  // ((w0 + w1) + w2) + w3 from 0.f: the former red[0] + red[1] + red[2] + red[3]
  }
  const int d = blockIdx.y * 64 + lane;
  if (d >= D) return;
  const f16* dm = dmm + (int64_t)b * K;
  const f16* tc = txt_n + d;
  constexpr int U = 16;
  float s = 0.f;
  int k = 0;
  for (; k + U <= K; k += U) {
    float tv[U], mv[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      tv[u] = (float)tc[(int64_t)(k + u) * D];
      mv[u] = (float)dm[k + u];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) s += mv[u] * tv[u];
  }
  for (; k < K; ++k) s += (float)dm[k] * (float)tc[(int64_t)k * D];
  const float v = r16((float)trow[d] / nv);
  const float a = (float)irow[d];
  const float cosg = dcos * v / nu - a * dotp / (nu * nu * nu);
  dimg_n[(int64_t)b * D + d] = (f16)(r16(s) + r16(cosg));
}

// d txt_n[k,:] = fp16( fp16(sum_b dmm[b,k] img_n[b,:]) + sum_{b: y_b = k} cos-path ) ; block per k
__global__ void dtxt_kernel(const f16* __restrict__ dmm, const f16* __restrict__ img_n, const f16* __restrict__ txt_n,
                            const int64_t* __restrict__ label, const float* __restrict__ cos_norms, int B, int K,
                            int D, f16* __restrict__ dtxt_n) {
  const int k = blockIdx.x;
  const float dcos = r16(-0.5f / (float)B);
  __shared__ float red[4];
  __shared__ float dots[64];
  // per matching b: g_v . txt_n[k]
  for (int b = 0; b < B; ++b) {
    if ((int)label[b] != k) continue;  // uniform across the block
    const float nu = cos_norms[2 * b];
    float dotp = 0.f;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
      float u = r16((float)img_n[(int64_t)b * D + d] / nu);
      dotp += dcos * u * (float)txt_n[(int64_t)k * D + d];
    }
    dotp = wave_sum(dotp);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = dotp;
    __syncthreads();
    if (threadIdx.x == 0) dots[b] = red[0] + red[1] + red[2] + red[3];
  }
  __syncthreads();
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += (float)dmm[(int64_t)b * K + k] * (float)img_n[(int64_t)b * D + d];
    float cg = 0.f;
    const float t = (float)txt_n[(int64_t)k * D + d];
    for (int b = 0; b < B; ++b) {
      if ((int)label[b] != k) continue;
      const float nu = cos_norms[2 * b], nv = cos_norms[2 * b + 1];
      const float u = r16((float)img_n[(int64_t)b * D + d] / nu);
      cg += dcos * u / nv - t * dots[b] / (nv * nv * nv);
    }
    dtxt_n[(int64_t)k * D + d] = (f16)(r16(s) + (cg != 0.f ? r16(cg) : 0.f));
  }
}


// ---- soft labels (trainers/maple.py:356-360) -------------------------------------------------------
// text_features_for_images = q @ txt_n: tgt[b,:] = fp16(sum_k fp16(q[b,k]) txt_n[k,:]), fp32 accumulate.
// The reference multiplies an fp32 label by the fp16 text features, which torch refuses
// ("expected m1 and m2 to have the same dtype") in its fp16 configuration; the label is taken in the
// text features' dtype, which is also what the product computes under torch.autocast.  Block per b.
__global__ void soft_target_kernel(const float* __restrict__ q, const f16* __restrict__ txt_n, int K, int D,
                                   f16* __restrict__ tgt) {
  const int b = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f;
    for (int k = 0; k < K; ++k) s += r16(q[(int64_t)b * K + k]) * (float)txt_n[(int64_t)k * D + d];
    tgt[(int64_t)b * D + d] = (f16)s;
  }
}

// Single block of 1024 threads, wave w handles rows b = w, w+16, ...
//   log_probs = fp16(log_softmax(logits)); t = max(q, 1e-8)
//   KL = sum_{b,k} t (log t - log_probs) / B  in fp32 (F.kl_div(..., "batchmean") of an fp16 input and an
//   fp32 target promotes to fp32); its input gradient fp16(-t/B) goes through the log_softmax backward:
//   dlogits = fp16(g - exp(log_probs) * sum_k g), dmm = fp16(dlogits * scale).
//   cos_b = cos(img_n[b], tgt[b]) as loss_kernel; its gradient w.r.t. tgt[b] (fp16) is written to gtgt.
// loss_out: [0] total = KL + fp16(0.5 * align) (fp32), [1] KL, [2] align, [3] nonfinite flag
__global__ void loss_soft_kernel(const f16* __restrict__ logits, const f16* __restrict__ img_n,
                                 const f16* __restrict__ tgt, const float* __restrict__ q, int B, int K, int D,
                                 const float* __restrict__ logit_scale, f16* __restrict__ dmm,
                                 f16* __restrict__ gtgt, float* __restrict__ cos_out, float* __restrict__ loss_out) {
  __shared__ float s_kl[64], s_cos[64];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const float sc = fminf(expf(logit_scale[0]), 100.f);
  const float invB = 1.0f / (float)B;
  const float dcos = r16(-0.5f * invB);
  for (int b = w; b < B; b += nw) {
    const f16* lr = logits + (int64_t)b * K;
    const float* qr = q + (int64_t)b * K;
    float mx = -INFINITY;
    for (int k = lane; k < K; k += 64) mx = fmaxf(mx, (float)lr[k]);
    mx = wave_max(mx);
    float se = 0.f;
    for (int k = lane; k < K; k += 64) se += expf((float)lr[k] - mx);
    se = wave_sum(se);
    const float lse = logf(se);
    float kl = 0.f, sg = 0.f;
    for (int k = lane; k < K; k += 64) {
      const float logp = r16((float)lr[k] - mx - lse);
      const float t = fmaxf(qr[k], 1e-8f);
      kl += t * (logf(t) - logp);
      sg += r16(-t * invB);
    }
    kl = wave_sum(kl);
    sg = wave_sum(sg);
    for (int k = lane; k < K; k += 64) {
      const float logp = r16((float)lr[k] - mx - lse);
      const float g = r16(-fmaxf(qr[k], 1e-8f) * invB);
      const float dl = r16(g - expf(logp) * sg);
      dmm[(int64_t)b * K + k] = (f16)mul32(dl, sc);
    }
    const f16* tr = tgt + (int64_t)b * D;
    const f16* ir = img_n + (int64_t)b * D;
    float su = 0.f, sv = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float a = (float)ir[d], t = (float)tr[d];
      su += a * a;
      sv += t * t;
    }
    const float nu = fmaxf(r16(sqrtf(wave_sum(su))), 1e-8f), nv = fmaxf(r16(sqrtf(wave_sum(sv))), 1e-8f);
    float c = 0.f, dotp = 0.f;
    for (int d = lane; d < D; d += 64) {
      const float a = r16((float)ir[d] / nu), t = r16((float)tr[d] / nv);
      c += r16(a * t);
      dotp += dcos * a * (float)tr[d];
    }
    c = r16(wave_sum(c));
    dotp = wave_sum(dotp);
    // d tgt[b,:] = dcos * u / nv - tgt * (dcos u . tgt) / nv^3   (the txt side of dtxt_kernel's cos path)
    for (int d = lane; d < D; d += 64) {
      const float a = r16((float)ir[d] / nu);
      gtgt[(int64_t)b * D + d] = (f16)(dcos * a / nv - (float)tr[d] * dotp / (nv * nv * nv));
    }
    if (lane == 0) {
      s_kl[b] = kl;
      s_cos[b] = c;
      cos_out[2 * b] = nu;
      cos_out[2 * b + 1] = nv;
    }
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float kl = 0.f, cs = 0.f;
    for (int b = 0; b < B; ++b) {
      kl += s_kl[b];
      cs += s_cos[b];
    }
    kl = kl / (float)B;
    const float align = r16(1.f - r16(cs / (float)B));
    const float total = kl + r16(0.5f * align);
    loss_out[0] = total;
    loss_out[1] = kl;
    loss_out[2] = align;
    loss_out[3] = isfinite(total) ? 0.f : 1.f;
  }
}

// d txt_n[k,:] = fp16( fp16(sum_b dmm[b,k] img_n[b,:]) + fp16(sum_b fp16(q[b,k]) gtgt[b,:]) ): the logits
// product's gradient plus the q @ txt_n product's (q^T . d tgt); block per k
__global__ void dtxt_soft_kernel(const f16* __restrict__ dmm, const f16* __restrict__ img_n,
                                 const float* __restrict__ q, const f16* __restrict__ gtgt, int B, int K, int D,
                                 f16* __restrict__ dtxt_n) {
  const int k = blockIdx.x;
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float s = 0.f, cg = 0.f;
    for (int b = 0; b < B; ++b) {
      s += (float)dmm[(int64_t)b * K + k] * (float)img_n[(int64_t)b * D + d];
      cg += r16(q[(int64_t)b * K + k]) * (float)gtgt[(int64_t)b * D + d];
    }
    dtxt_n[(int64_t)k * D + d] = (f16)(r16(s) + r16(cg));
  }
}

// normalize backward: dx = fp16(dy/n - x * (dy . x) / n^3)   ; one wave per row
__global__ void normalize_bwd_kernel(const f16* __restrict__ x, const f16* __restrict__ dy,
                                     const float* __restrict__ norm, f16* __restrict__ dx, int rows, int D) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (row >= rows) return;
  const float n = norm[row];
  float s = 0.f;
  for (int d = lane; d < D; d += 64) s += (float)dy[(int64_t)row * D + d] * (float)x[(int64_t)row * D + d];
  s = wave_sum(s);
  for (int d = lane; d < D; d += 64) {
    const float g = (float)dy[(int64_t)row * D + d] / n - (float)x[(int64_t)row * D + d] * s / (n * n * n);
    dx[(int64_t)row * D + d] = (f16)g;
  }
}

// eval argmax (trainers/maple.py:674-677): pred[b] = argmax_k logits[b,k] (first maximum, NaN counts as
// the maximum like torch.argmax); acc[0] += #(pred == label), acc[1] += B.  One wave per row.
__global__ void argmax_correct_kernel(const f16* __restrict__ logits, int B, int K, const int64_t* __restrict__ label,
                                      int64_t* __restrict__ pred, float* __restrict__ acc) {
  __shared__ int s_ok[16];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  int ok = 0;
  for (int b = w; b < B; b += 16) {
    float best = -INFINITY;
    int bi = -1;  // no candidate yet
    for (int k = lane; k < K; k += 64) {  // ascending k: on ties the first index stays
      const float v = (float)logits[(int64_t)b * K + k];
      const bool better = bi < 0 || (isnan(v) ? !isnan(best) : (!isnan(best) && v > best));
      if (better) {
        best = v;
        bi = k;
      }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
      const float ob = __shfl_xor(best, o, 64);
      const int oi = __shfl_xor(bi, o, 64);
      bool take;
      if (oi < 0)
        take = false;
      else if (bi < 0)
        take = true;
      else if (isnan(ob) || isnan(best))
        take = isnan(ob) && (!isnan(best) || oi < bi);
      else
        take = ob > best || (ob == best && oi < bi);
      if (take) {
        best = ob;
        bi = oi;
      }
    }
    if (lane == 0) {
      if (pred) pred[b] = bi;
      if (label) ok += (bi == (int)label[b]);
    }
  }
  if (lane == 0) s_ok[w] = ok;
  __syncthreads();
  if (threadIdx.x == 0 && acc) {
    int tot = 0;
    for (int i = 0; i < 16; ++i) tot += s_ok[i];
    acc[0] += (float)tot;
    acc[1] += (float)B;
  }
}

}  // namespace

extern "C" int mf_argmax_correct(const void* logits, int B, int K, const int64_t* label, int64_t* pred, float* acc,
                                 void* stream) {
  if (B <= 0) return 0;
  argmax_correct_kernel<<<1, 1024, 0, (hipStream_t)stream>>>((const f16*)logits, B, K, label, pred, acc);
  MF_CHECK_LAUNCH();
  return 0;
}

// workspace floats needed: 2*B (cos norms) + (B+K) (feature norms)
extern "C" int mf_clip_head_fwd(const void* img, const void* txt, int B, int K, int D, const float* logit_scale,
                                void* img_n, void* txt_n, float* norms, void* mm, void* logits, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  normalize_rows_kernel<<<(B + 3) / 4, 256, 0, st>>>((const f16*)img, (f16*)img_n, norms, B, D);
  normalize_rows_kernel<<<(K + 3) / 4, 256, 0, st>>>((const f16*)txt, (f16*)txt_n, norms + B, K, D);
  const int64_t threads = (int64_t)B * K * 64;
  logits_kernel<<<(unsigned)((threads + 255) / 256), 256, 0, st>>>((const f16*)img_n, (const f16*)txt_n, B, K, D,
                                                                   logit_scale, (f16*)mm, (f16*)logits);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_clip_loss_fwd_bwd(const void* img, const void* txt, const void* img_n, const void* txt_n,
                                    const float* norms, const void* logits, const int64_t* label, int B, int K, int D,
                                    const float* logit_scale, void* dmm, float* cos_ws, float* loss_out,
                                    void* dimg_n, void* dtxt_n, void* dimg, void* dtxt, void* stream) {
  if (B > 64) return mf_set_error("mf_clip_loss_fwd_bwd: B <= 64", -1);
  hipStream_t st = (hipStream_t)stream;
  loss_kernel<<<1, 1024, 0, st>>>((const f16*)logits, (const f16*)img_n, (const f16*)txt_n, label, B, K, D,
                                 logit_scale, (f16*)dmm, cos_ws, loss_out);
  dimg_kernel<<<dim3(B, (D + 63) / 64), 64, 0, st>>>((const f16*)dmm, (const f16*)img_n, (const f16*)txt_n, label, nullptr, cos_ws, B,
                                 K, D, (f16*)dimg_n);
  dtxt_kernel<<<K, 256, 0, st>>>((const f16*)dmm, (const f16*)img_n, (const f16*)txt_n, label, cos_ws, B, K, D,
                                 (f16*)dtxt_n);
  normalize_bwd_kernel<<<(B + 3) / 4, 256, 0, st>>>((const f16*)img, (const f16*)dimg_n, norms, (f16*)dimg, B, D);
  normalize_bwd_kernel<<<(K + 3) / 4, 256, 0, st>>>((const f16*)txt, (const f16*)dtxt_n, norms + B, (f16*)dtxt, K, D);
  MF_CHECK_LAUNCH();
  return 0;
}

// soft_ws: 2*B*D fp16 (the targets q @ txt_n and their gradient)
extern "C" int mf_clip_loss_soft_fwd_bwd(const void* img, const void* txt, const void* img_n, const void* txt_n,
                                         const float* norms, const void* logits, const float* label_probs, int B,
                                         int K, int D, const float* logit_scale, void* dmm, float* cos_ws,
                                         void* soft_ws, float* loss_out, void* dimg_n, void* dtxt_n, void* dimg,
                                         void* dtxt, void* stream) {
  if (B > 64) return mf_set_error("mf_clip_loss_soft_fwd_bwd: B <= 64", -1);
  hipStream_t st = (hipStream_t)stream;
  f16* tgt = (f16*)soft_ws;
  f16* gtgt = tgt + (int64_t)B * D;
  soft_target_kernel<<<B, 256, 0, st>>>(label_probs, (const f16*)txt_n, K, D, tgt);
  loss_soft_kernel<<<1, 1024, 0, st>>>((const f16*)logits, (const f16*)img_n, tgt, label_probs, B, K, D, logit_scale,
                                      (f16*)dmm, gtgt, cos_ws, loss_out);
  dimg_kernel<<<dim3(B, (D + 63) / 64), 64, 0, st>>>((const f16*)dmm, (const f16*)img_n, (const f16*)txt_n, nullptr, tgt, cos_ws, B, K, D,
                                 (f16*)dimg_n);
  dtxt_soft_kernel<<<K, 256, 0, st>>>((const f16*)dmm, (const f16*)img_n, label_probs, gtgt, B, K, D,
                                      (f16*)dtxt_n);
  normalize_bwd_kernel<<<(B + 3) / 4, 256, 0, st>>>((const f16*)img, (const f16*)dimg_n, norms, (f16*)dimg, B, D);
  normalize_bwd_kernel<<<(K + 3) / 4, 256, 0, st>>>((const f16*)txt, (const f16*)dtxt_n, norms + B, (f16*)dtxt, K, D);
  MF_CHECK_LAUNCH();
  return 0;
}
