// Shared helpers for the MI355X (gfx950 / CDNA4) kernels of the federated MaPLe path.
// Everything here is device-side plumbing: vector types for MFMA fragments, fp16 rounding
// helpers that pin the reference's rounding points, wave64 reductions and the C-ABI status
// convention (int status, mf_last_error()).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef _Float16 f16;
typedef f16 f16x2 __attribute__((ext_vector_type(2)));
typedef f16 f16x4 __attribute__((ext_vector_type(4)));
typedef f16 f16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4 __attribute__((ext_vector_type(4)));

#define MF_DEV __device__ __forceinline__

// Round-to-nearest-even fp32 -> fp16 -> fp32: the rounding every fp16 torch op applies once
// to its opmath (fp32) result.
MF_DEV float r16(float x) { return (float)(f16)x; }

MF_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
MF_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// QuickGELU with the reference's three fp16 roundings (clip/model.py:162-164):
//   t1 = fp16(1.702*f); t2 = fp16(sigmoid(t1)); g = fp16(f*t2)
// sigmoid in fp32 with the hardware reciprocal (v_rcp_f32, 1 ulp): its result is rounded to fp16
// next, so the fp32 ulp matters only within 2^-13 of an fp16 rounding boundary.  t1 and the backward's
// fp16(dt1*1.702) are left to the compiler's v_fma_mixlo_f16, which rounds the exact product once (the
// reference: fp32 product, then fp16): 61 of the 61 094 finite fp16 f give a t1 one fp16 ulp away.  r06 measured the
// reference's two roundings there (mul32 below): logits moved both ways (c3_j9_k10_b4: max |err| vs the reference
// 2.93e-3 -> 4.88e-3 against a 4.0e-3 gate, vs fp64 3.5e-3 -> 2.5e-3), so the gated form stays.
MF_DEV float sigmoid32(float t) { return __builtin_amdgcn_rcpf(1.0f + __expf(-t)); }

// fp32 product of a and b, materialised as fp32 before any fp16 rounding of it: the reference's fp16 op rounds its
// fp32 opmath product to fp16 (two roundings), while the compiler folds fp16(a * b) into v_fma_mixlo_f16, which
// rounds the exact product once -- a different fp16 for 61 of the 61 094 finite fp16 inputs of f * 1.702f
// (r06, tests/diagnostics/mixround/).  Products of two fp16 values are exact in fp32 and need no barrier.  Used
// where an fp16 tensor meets an fp32 scalar at the head and in the optimizer (logit scale, clip coefficient,
// momentum).
MF_DEV float mul32(float a, float b) {
  float p = a * b;
  asm volatile("" : "+v"(p));
  return p;
}

MF_DEV float quick_gelu16(float f, float* t2_out) {
  float t1 = r16(f * 1.702f);
  float t2 = r16(sigmoid32(t1));
  *t2_out = t2;
  return r16(f * t2);
}
// Its autograd backward (mul / sigmoid / mul nodes, then fp16 accumulation of the two uses of f):
//   da = fp16(dg*t2); dt2 = fp16(dg*f); db = fp16(dt1*1.702); df = fp16(da+db), where torch's CPU
//   sigmoid_backward for Half runs in fp16 arithmetic op by op (measured against
//   aten::sigmoid_backward): dt1 = fp16(fp16(dt2*fp16(1-t2))*t2)
MF_DEV float quick_gelu16_bwd(float dg, float f) {
  float t1 = r16(f * 1.702f);
  float t2 = r16(sigmoid32(t1));
  float da = r16(dg * t2);
  float dt2 = r16(dg * f);
  float dt1 = r16(r16(dt2 * r16(1.0f - t2)) * t2);
  float db = r16(dt1 * 1.702f);
  return r16(da + db);
}

// Deterministic column reduction of `nblk` partial rows: out[c] (=|+=) sum_b part[b*ld + c].
// One 1024-thread block per 64 columns: 16 row groups x 64 lanes, each lane summing its group's rows
// with 4 independent loads in flight, then a fixed-order LDS reduction over the 16 groups (the same
// order on every launch -> bitwise reproducible).  Up to two (part, out) pairs per launch
// (blockIdx.y selects the pair: LayerNorm dgamma and dbeta in one launch).
namespace {
template <bool OUT16>
__global__ __launch_bounds__(1024) void col_reduce_kernel(const float* __restrict__ part0,
                                                          const float* __restrict__ part1, int nblk, int C,
                                                          int64_t ld, void* out0, void* out1, int accumulate) {
  __shared__ float red[16][65];
  const float* part = blockIdx.y ? part1 : part0;
  void* out = blockIdx.y ? out1 : out0;
  const int lane = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane;
  float s0 = 0.f, s1 = 0.f, s2 = 0.f, s3 = 0.f;
  if (c < C) {
    int b = g;
    for (; b + 48 < nblk; b += 64) {
      s0 += part[(int64_t)b * ld + c];
      s1 += part[(int64_t)(b + 16) * ld + c];
      s2 += part[(int64_t)(b + 32) * ld + c];
      s3 += part[(int64_t)(b + 48) * ld + c];
    }
    for (; b < nblk; b += 16) s0 += part[(int64_t)b * ld + c];
  }
  red[g][lane] = (s0 + s1) + (s2 + s3);
  __syncthreads();
  if (g == 0 && c < C) {
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < 16; ++k) s += red[k][lane];
    if (OUT16) {
      f16* o = (f16*)out + c;
      *o = accumulate ? (f16)((float)*o + s) : (f16)s;
    } else {
      float* o = (float*)out + c;
      *o = accumulate ? *o + s : s;
    }
  }
}
}  // namespace

#define MF_CHECK_LAUNCH()                                                     \
  do {                                                                        \
    hipError_t _e = hipGetLastError();                                        \
    if (_e != hipSuccess) return mf_set_error(hipGetErrorString(_e), (int)_e); \
  } while (0)

extern "C" int mf_set_error(const char* msg, int code);

// Compute units of the current device (256 on an MI355X; fewer under a compute partition mode), cached per device.
inline int mf_cu_count() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] <= 0) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cached[dev] = n;
  }
  return cached[dev];
}
