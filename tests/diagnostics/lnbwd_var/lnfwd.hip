// Diagnostic (GPU box): ln_fwd2_kernel<768, 1> (csrc/layernorm.hip) at the c4 vision shape, and candidates:
//   MODE 0: the library's arithmetic and access pattern (one row per half-wave, gamma / beta from global per row)
//   MODE 1: gamma / beta staged once per workgroup into LDS (6 KB) and read from there
//   MODE 2: gamma = 1, beta = 0 (timing only)
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

template <int MODE>
__global__ __launch_bounds__(256) void lnf_kernel(const f16* __restrict__ x, const float* __restrict__ gamma,
                                                  const float* __restrict__ beta, f16* __restrict__ y,
                                                  float* __restrict__ mean_out, float* __restrict__ rstd_out, int rows) {
  constexpr int D = 768, CH = 3;
  __shared__ __attribute__((aligned(16))) float sg[MODE == 1 ? D : 1], sb[MODE == 1 ? D : 1];
  const int hl = threadIdx.x & 31;
  const int row = blockIdx.x * 8 + (threadIdx.x >> 5);
  if (MODE == 1) {
    for (int i = threadIdx.x; i < D / 4; i += 256) {
      *(f32x4*)(sg + 4 * i) = *(const f32x4*)(gamma + 4 * i);
      *(f32x4*)(sb + 4 * i) = *(const f32x4*)(beta + 4 * i);
    }
  }
  f16x8 t[CH];
  const int rr = row < rows ? row : rows - 1;
#pragma unroll
  for (int j = 0; j < CH; ++j) t[j] = *(const f16x8*)(x + (int64_t)rr * D + 8 * (hl + 32 * j));
  if (MODE == 1) __syncthreads();
  if (row >= rows) return;
  float v[CH * 8];
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int j = 0; j < CH; ++j)
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      v[j * 8 + e] = (float)t[j][e];
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
  f16* yr = y + (int64_t)row * D;
#pragma unroll
  for (int j = 0; j < CH; ++j) {
    const int c = 8 * (hl + 32 * j);
    f32x4 g0, g1, b0, b1;
    if (MODE == 2) {
      g0 = g1 = (f32x4){1.f, 1.f, 1.f, 1.f};
      b0 = b1 = (f32x4){0.f, 0.f, 0.f, 0.f};
    } else if (MODE == 1) {
      g0 = *(const f32x4*)(sg + c), g1 = *(const f32x4*)(sg + c + 4);
      b0 = *(const f32x4*)(sb + c), b1 = *(const f32x4*)(sb + c + 4);
    } else {
      g0 = *(const f32x4*)(gamma + c), g1 = *(const f32x4*)(gamma + c + 4);
      b0 = *(const f32x4*)(beta + c), b1 = *(const f32x4*)(beta + c + 4);
    }
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
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}
}  // namespace

extern "C" int lnf_launch(int mode, const void* x, const float* gamma, const float* beta, void* y, float* mean,
                          float* rstd, int rows, void* stream) {
  const dim3 g((rows + 7) / 8);
  hipStream_t st = (hipStream_t)stream;
  switch (mode) {
    case 0: lnf_kernel<0><<<g, 256, 0, st>>>((const f16*)x, gamma, beta, (f16*)y, mean, rstd, rows); break;
    case 1: lnf_kernel<1><<<g, 256, 0, st>>>((const f16*)x, gamma, beta, (f16*)y, mean, rstd, rows); break;
    case 2: lnf_kernel<2><<<g, 256, 0, st>>>((const f16*)x, gamma, beta, (f16*)y, mean, rstd, rows); break;
    default: return -1;
  }
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
