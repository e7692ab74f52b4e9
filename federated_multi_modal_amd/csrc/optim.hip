// Optimizer step and federated averaging over the flat trainable buffers.
//
// The trainable tensors (trainers/maple.py:447-479) live in two flat device buffers, one fp16 and
// one fp32, each tensor a contiguous segment; grads and SGD momentum mirror them.  That turns
//   torch.nn.utils.clip_grad_norm_(params, 1.0)      (trainers/maple.py:592-596)
//   Dassl SGD(momentum 0.9, wd 5e-4).step()           (trainers/maple.py:598)
//   safe_average_weights / check_weights_valid        (trainers/maple_fed.py:309-325)
// into a handful of streaming kernels with no host synchronisation: the clip coefficient stays on
// the device and the SGD kernel reads it.
//
// Rounding points follow torch: per-tensor norms in the grad's dtype (fp16 norm for fp16 grads),
// total norm in fp32, coef = clamp(1/(total+1e-6), max 1); g = T(g*coef); d_p = T(g + wd*p);
// buf = d_p (first step) or T(T(buf*mom) + d_p); p = T(p - lr*buf).
#include <type_traits>

#include "mf_common.h"

#pragma clang fp contract(off)

namespace {

constexpr int CHUNK = 8192;

struct Chunk {
  int seg;
  int is16;
  int64_t start, end;  // element range inside the segment's flat buffer
};

__global__ void sumsq_chunks_kernel(const f16* __restrict__ g16, const float* __restrict__ g32,
                                    const Chunk* __restrict__ chunks, float* __restrict__ part) {
  const Chunk c = chunks[blockIdx.x];
  float s = 0.f;
  // 16-byte loads over the chunk's 16-byte-aligned middle (the flat buffers are 256-B aligned), element
  // loads for the ragged head and tail
  if (c.is16) {
    const int64_t a = min(c.end, (c.start + 7) & ~(int64_t)7), b = max(a, c.end & ~(int64_t)7);
    for (int64_t i = c.start + threadIdx.x; i < a; i += blockDim.x) {
      float v = (float)g16[i];
      s += v * v;
    }
    for (int64_t i = a / 8 + threadIdx.x; i < b / 8; i += blockDim.x) {
      const f16x8 v = ((const f16x8*)g16)[i];
#pragma unroll
      for (int e = 0; e < 8; ++e) s += (float)v[e] * (float)v[e];
    }
    for (int64_t i = b + threadIdx.x; i < c.end; i += blockDim.x) {
      float v = (float)g16[i];
      s += v * v;
    }
  } else {
    const int64_t a = min(c.end, (c.start + 3) & ~(int64_t)3), b = max(a, c.end & ~(int64_t)3);
    for (int64_t i = c.start + threadIdx.x; i < a; i += blockDim.x) {
      float v = g32[i];
      s += v * v;
    }
    for (int64_t i = a / 4 + threadIdx.x; i < b / 4; i += blockDim.x) {
      const f32x4 v = ((const f32x4*)g32)[i];
      s += v[0] * v[0] + v[1] * v[1] + v[2] * v[2] + v[3] * v[3];
    }
    for (int64_t i = b + threadIdx.x; i < c.end; i += blockDim.x) {
      float v = g32[i];
      s += v * v;
    }
  }
  __shared__ float red[4];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// One block of 1024 threads: per-segment norms from the per-chunk partial sums (the chunks of a
// segment are consecutive), total norm, clip coefficient.  The chunk list is walked in tiles of 1024
// with a segmented inclusive scan (Hillis-Steele in LDS, fixed order -> deterministic); the last
// chunk of each segment yields that segment's sum of squares (plus the carry of a segment that
// started in an earlier tile).  torch.nn.utils.clip_grad_norm_: per-tensor norms in the grad's dtype
// (fp16 tensors round their norm to fp16), total = ||(norm_t)_t||_2 in fp32,
// coef = clamp(max_norm / (total + 1e-6), max 1).
// out[0] = total norm, out[1] = clip coef, out[2] = 1 if total is finite else 0
__global__ __launch_bounds__(1024) void clip_coef_kernel(const float* __restrict__ part,
                                                         const Chunk* __restrict__ chunks, int nchunks,
                                                         float max_norm, float* __restrict__ out,
                                                         float* __restrict__ hyper = nullptr,
                                                         const float* __restrict__ halt_src = nullptr,
                                                         const int* __restrict__ halt_src2 = nullptr) {
  __shared__ float sv[1024];
  __shared__ int sseg[1024];
  __shared__ float red[16];
  __shared__ float carry_val;
  __shared__ int carry_seg;
  const int t = threadIdx.x;
  if (t == 0) {
    carry_val = 0.f;
    carry_seg = -1;
  }
  float acc = 0.f;
  for (int base = 0; base < nchunks; base += 1024) {
    const int c = base + t;
    const int seg = c < nchunks ? chunks[c].seg : -1;
    float v = c < nchunks ? part[c] : 0.f;
    sseg[t] = seg;
    sv[t] = v;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
      float add = 0.f;
      if (t >= off && sseg[t - off] == seg) add = sv[t - off];
      __syncthreads();
      v += add;
      sv[t] = v;
      __syncthreads();
    }
    const bool last = c < nchunks && (c == nchunks - 1 || chunks[c + 1].seg != seg);
    if (last) {
      float ss = v;
      if (seg == carry_seg && sseg[0] == seg) ss += carry_val;  // segment began in an earlier tile
      float nrm = sqrtf(ss);
      if (chunks[c].is16) nrm = r16(nrm);
      acc += nrm * nrm;
    }
    __syncthreads();
    if (t == 1023) {
      const float prev = (seg == carry_seg && sseg[0] == seg) ? carry_val : 0.f;
      carry_val = v + prev;
      carry_seg = seg;
    }
    __syncthreads();
  }
  acc = wave_sum(acc);
  if ((t & 63) == 0) red[t >> 6] = acc;
  __syncthreads();
  if (t == 0) {
    float tot = 0.f;
    for (int i = 0; i < 16; ++i) tot += red[i];
    const float total = sqrtf(tot);
    float coef = max_norm / (total + 1e-6f);
    coef = coef > 1.f ? 1.f : coef;
    out[0] = total;
    out[1] = coef;
    out[2] = isfinite(total) ? 1.f : 0.f;
    // the step's halt latch (torch.maximum(hyper[4], loss non-finite flag)) for the SGD launch that follows
    if (hyper) {
      const float h = fmaxf(hyper[4], halt_src[0]);
      hyper[4] = halt_src2 ? fmaxf(h, (float)halt_src2[0]) : h;
    }
  }
}

// hyper = {lr, momentum, weight_decay, first_step (1.0 = momentum buffer not yet created), halt}: read from
// device memory so a captured step replays with the current schedule value.  halt != 0 (a non-finite loss
// earlier in the epoch or in this step) leaves parameters, gradients and momentum untouched: the reference
// raises at the first non-finite loss before its backward (trainers/maple.py:375-376), so no update follows.
template <typename T>
__global__ void sgd_kernel(T* __restrict__ p, T* __restrict__ g, T* __restrict__ buf, int64_t n,
                           const float* __restrict__ coef_ptr, const float* __restrict__ hyper) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || hyper[4] != 0.f) return;
  const float coef = coef_ptr[1];
  const float lr = hyper[0], momentum = hyper[1], wd = hyper[2];
  const bool first = hyper[3] != 0.f;
  const float pv = (float)p[i];
  const float gc = (float)(T)mul32((float)g[i], coef);
  g[i] = (T)gc;
  const float dp = (float)(T)(gc + wd * pv);
  float b;
  if (first)
    b = dp;
  else
    b = (float)(T)((float)(T)mul32((float)buf[i], momentum) + dp);
  buf[i] = (T)b;
  p[i] = (T)(pv + (-lr) * b);
}

// sgd_kernel on 8 consecutive elements per thread (16-byte fp16 / 2 x 16-byte fp32 accesses), the same
// per-element arithmetic; n % 8 == 0 and 16-byte aligned buffers
template <typename T>
MF_DEV void sgd8_body(T* __restrict__ p, T* __restrict__ g, T* __restrict__ buf, int64_t n8, int64_t i,
                      const float* __restrict__ coef_ptr, const float* __restrict__ hyper) {
  using V = typename std::conditional<std::is_same<T, f16>::value, f16x8, float __attribute__((ext_vector_type(8)))>::type;
  if (i >= n8 || hyper[4] != 0.f) return;
  const float coef = coef_ptr[1];
  const float lr = hyper[0], momentum = hyper[1], wd = hyper[2];
  const bool first = hyper[3] != 0.f;
  V pv = ((V*)p)[i], gv = ((V*)g)[i], bv = first ? V{} : ((V*)buf)[i];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const float pe = (float)pv[e];
    const float gc = (float)(T)mul32((float)gv[e], coef);
    gv[e] = (T)gc;
    const float dp = (float)(T)(gc + wd * pe);
    float b;
    if (first)
      b = dp;
    else
      b = (float)(T)((float)(T)mul32((float)bv[e], momentum) + dp);
    bv[e] = (T)b;
    pv[e] = (T)(pe + (-lr) * b);
  }
  ((V*)g)[i] = gv;
  ((V*)buf)[i] = bv;
  ((V*)p)[i] = pv;
}

template <typename T>
__global__ void sgd8_kernel(T* __restrict__ p, T* __restrict__ g, T* __restrict__ buf, int64_t n8,
                            const float* __restrict__ coef_ptr, const float* __restrict__ hyper) {
  sgd8_body<T>(p, g, buf, n8, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, coef_ptr, hyper);
}

// both flat buffers' SGD in one launch: blocks [0, nb16) update the fp16 trainables, the rest the fp32 ones
__global__ void sgd8_both_kernel(f16* __restrict__ p16, f16* __restrict__ g16, f16* __restrict__ b16, int64_t n16_8,
                                 float* __restrict__ p32, float* __restrict__ g32, float* __restrict__ b32,
                                 int64_t n32_8, unsigned nb16, const float* __restrict__ coef_ptr,
                                 const float* __restrict__ hyper) {
  if (blockIdx.x < nb16)
    sgd8_body<f16>(p16, g16, b16, n16_8, (int64_t)blockIdx.x * blockDim.x + threadIdx.x, coef_ptr, hyper);
  else
    sgd8_body<float>(p32, g32, b32, n32_8, (int64_t)(blockIdx.x - nb16) * blockDim.x + threadIdx.x, coef_ptr, hyper);
}

// bucket[0:n16] = float(p16), bucket[n16:n16+n32] = p32
__global__ void pack_kernel(const f16* __restrict__ p16, int64_t n16, const float* __restrict__ p32, int64_t n32,
                            const int* __restrict__ invalid, float* __restrict__ bucket) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool bad = invalid && invalid[0] != 0;  // this client's weights are excluded (maple_fed.py:272-277)
  if (i < n16)
    bucket[i] = bad ? 0.f : (float)p16[i];
  else if (i < n16 + n32)
    bucket[i] = bad ? 0.f : p32[i - n16];
  else if (i == n16 + n32)
    bucket[i] = bad ? 0.f : 1.f;  // this client's vote in the valid-client count
}
// mean = sum / n_valid with n_valid = bucket[n16+n32] read on the device (no host sync); value =
// fp16(mean); p16 = value, p32 = float(value)   (the `.half()` of trainers/maple_fed.py:314 followed
// by load_state_dict into each parameter's dtype), and the value is kept as the new global copy
// (g16/g32).  n_valid == 0 -> every client failed: the round is skipped and every client goes back
// to the previous global weights (trainers/maple_fed.py:288-290 + the next round's broadcast).
__global__ void unpack_kernel(const float* __restrict__ bucket, f16* __restrict__ p16, int64_t n16,
                              float* __restrict__ p32, int64_t n32, f16* __restrict__ g16, float* __restrict__ g32) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const float n_valid = bucket[n16 + n32];
  if (i < n16) {
    if (n_valid == 0.f) {
      if (g16) p16[i] = g16[i];
    } else {
      const f16 v = (f16)(bucket[i] / n_valid);
      p16[i] = v;
      if (g16) g16[i] = v;
    }
  } else if (i < n16 + n32) {
    const int64_t j = i - n16;
    if (n_valid == 0.f) {
      if (g32) p32[j] = g32[j];
    } else {
      const float v = r16(bucket[i] / n_valid);
      p32[j] = v;
      if (g32) g32[j] = v;
    }
  }
}

// out[i] = (((g_0[i] + g_1[i]) + g_2[i]) + ...) in client order, g_c = gathered + c * stride: the
// per-key torch.stack(...) sum of trainers/maple_fed.py:311-314 in the order the reference stacks its
// clients, whatever order the collective delivered them in (8 floats per thread, fp32 accumulation)
__global__ void reduce_ordered_kernel(const float* __restrict__ g, int nclients, int64_t stride, int64_t n,
                                      float* __restrict__ out) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i >= n) return;
  if (i + 4 <= n && stride % 4 == 0 && ((uintptr_t)g % 16) == 0 && ((uintptr_t)out % 16) == 0) {
    float4 acc = *(const float4*)(g + i);
    for (int c = 1; c < nclients; ++c) {
      const float4 v = *(const float4*)(g + (int64_t)c * stride + i);
      acc.x += v.x;
      acc.y += v.y;
      acc.z += v.z;
      acc.w += v.w;
    }
    *(float4*)(out + i) = acc;
  } else {
    for (int64_t j = i; j < n && j < i + 4; ++j) {
      float acc = g[j];
      for (int c = 1; c < nclients; ++c) acc += g[(int64_t)c * stride + j];
      out[j] = acc;
    }
  }
}

// flag[0] |= 1 if any element is NaN/Inf
__global__ void nonfinite_kernel(const void* __restrict__ x, int64_t n, int is16, int* __restrict__ flag) {
  int bad = 0;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float v = is16 ? (float)((const f16*)x)[i] : ((const float*)x)[i];
    bad |= !isfinite(v);
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

inline unsigned nblk(int64_t n, int b = 256) { return (unsigned)((n + b - 1) / b); }

}  // namespace

extern "C" int mf_optim_chunk_bytes() { return (int)sizeof(Chunk); }
extern "C" int mf_optim_chunk_elems() { return CHUNK; }

// chunks: device array of Chunk {int seg, int is16, int64 start, int64 end}; part: nchunks floats;
// out: 3 floats (total norm, coef, finite flag)
extern "C" int mf_clip_grad_norm(const void* g16, const float* g32, const void* chunks, int nchunks, float max_norm,
                                 float* part, float* out, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (nchunks <= 0) return 0;
  sumsq_chunks_kernel<<<nchunks, 256, 0, st>>>((const f16*)g16, g32, (const Chunk*)chunks, part);
  MF_CHECK_LAUNCH();
  clip_coef_kernel<<<1, 1024, 0, st>>>(part, (const Chunk*)chunks, nchunks, max_norm, out);
  MF_CHECK_LAUNCH();
  return 0;
}

// The whole optimizer step in three launches: clip_grad_norm_ (partial sums, then the coefficient, which also
// latches hyper[4] = max(hyper[4], *halt_src, *input_flag) -- the two torch.maximum launches the engine used to
// make, at the step's start for the input check and here for the loss), then SGD over the fp16 and the fp32 flat
// buffers in one launch.  Bit-identical to mf_clip_grad_norm + two mf_sgd_step.  input_flag may be null.
extern "C" int mf_sgd_step(void* p, void* g, void* buf, int64_t n, int is16, const float* coef, const float* hyper,
                           void* stream);
extern "C" int mf_optimizer_step(void* p16, void* g16, void* b16, int64_t n16, float* p32, float* g32, float* b32,
                                 int64_t n32, const void* chunks, int nchunks, float max_norm, float* part, float* out,
                                 float* hyper, const float* halt_src, const int* input_flag, void* stream) {
  hipStream_t st = (hipStream_t)stream;
  if (nchunks > 0) {
    sumsq_chunks_kernel<<<nchunks, 256, 0, st>>>((const f16*)g16, g32, (const Chunk*)chunks, part);
    MF_CHECK_LAUNCH();
  }
  clip_coef_kernel<<<1, 1024, 0, st>>>(part, (const Chunk*)chunks, nchunks, max_norm, out, hyper, halt_src,
                                       input_flag);
  MF_CHECK_LAUNCH();
  const bool vec16 = n16 % 8 == 0 && (uintptr_t)p16 % 32 == 0 && (uintptr_t)g16 % 32 == 0 && (uintptr_t)b16 % 32 == 0;
  const bool vec32 = n32 % 8 == 0 && (uintptr_t)p32 % 32 == 0 && (uintptr_t)g32 % 32 == 0 && (uintptr_t)b32 % 32 == 0;
  if (vec16 && vec32 && n16 + n32 > 0) {
    const unsigned nb16 = nblk(n16 / 8), nb32 = nblk(n32 / 8);
    sgd8_both_kernel<<<nb16 + nb32, 256, 0, st>>>((f16*)p16, (f16*)g16, (f16*)b16, n16 / 8, p32, g32, b32, n32 / 8,
                                                  nb16, out, hyper);
    MF_CHECK_LAUNCH();
    return 0;
  }
  int rc = mf_sgd_step(p16, g16, b16, n16, 1, out, hyper, stream);
  return rc ? rc : mf_sgd_step(p32, g32, b32, n32, 0, out, hyper, stream);
}

extern "C" int mf_sgd_step(void* p, void* g, void* buf, int64_t n, int is16, const float* coef,
                           const float* hyper, void* stream) {
  if (n <= 0) return 0;
  hipStream_t st = (hipStream_t)stream;
  const bool vec = n % 8 == 0 && (uintptr_t)p % 32 == 0 && (uintptr_t)g % 32 == 0 && (uintptr_t)buf % 32 == 0;
  if (vec && is16)
    sgd8_kernel<f16><<<nblk(n / 8), 256, 0, st>>>((f16*)p, (f16*)g, (f16*)buf, n / 8, coef, hyper);
  else if (vec)
    sgd8_kernel<float><<<nblk(n / 8), 256, 0, st>>>((float*)p, (float*)g, (float*)buf, n / 8, coef, hyper);
  else if (is16)
    sgd_kernel<f16><<<nblk(n), 256, 0, st>>>((f16*)p, (f16*)g, (f16*)buf, n, coef, hyper);
  else
    sgd_kernel<float><<<nblk(n), 256, 0, st>>>((float*)p, (float*)g, (float*)buf, n, coef, hyper);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_fedavg_pack(const void* p16, int64_t n16, const float* p32, int64_t n32, const int* invalid_flag,
                              float* bucket, void* stream) {
  if (n16 < 0 || n32 < 0) return mf_set_error("mf_fedavg_pack: negative size", -1);
  pack_kernel<<<nblk(n16 + n32 + 1), 256, 0, (hipStream_t)stream>>>((const f16*)p16, n16, p32, n32, invalid_flag,
                                                                    bucket);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_fedavg_unpack(const float* bucket, void* p16, int64_t n16, float* p32, int64_t n32, void* g16,
                                float* g32, void* stream) {
  if (n16 + n32 <= 0) return 0;
  unpack_kernel<<<nblk(n16 + n32), 256, 0, (hipStream_t)stream>>>(bucket, (f16*)p16, n16, p32, n32, (f16*)g16, g32);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_fedavg_reduce_ordered(const float* gathered, int nclients, int64_t stride, int64_t n, float* out,
                                        void* stream) {
  if (nclients < 1 || n < 0 || stride < n) return mf_set_error("mf_fedavg_reduce_ordered: bad sizes", -1);
  if (n == 0) return 0;
  reduce_ordered_kernel<<<nblk((n + 3) / 4), 256, 0, (hipStream_t)stream>>>(gathered, nclients, stride, n, out);
  MF_CHECK_LAUNCH();
  return 0;
}

extern "C" int mf_nonfinite_flag(const void* x, int64_t n, int is16, int* flag, void* stream) {
  if (n <= 0) return 0;
  unsigned g = nblk(n);
  if (g > 2048) g = 2048;
  nonfinite_kernel<<<g, 256, 0, (hipStream_t)stream>>>(x, n, is16, flag);
  MF_CHECK_LAUNCH();
  return 0;
}
