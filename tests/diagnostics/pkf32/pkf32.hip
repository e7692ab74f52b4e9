// Diagnostic only: do gfx950's packed fp32 VALU ops (v_pk_mul_f32 / v_pk_add_f32) compute what the scalar ones
// (v_mul_f32 / v_add_f32 / v_fma_f32) compute?  One thread per input pair (a[i], b[i]); out[6i..6i+5] = scalar
// mul, packed mul (low half), scalar add, packed add (low half), scalar fma(a, b, c), packed fma (low half), with
// c = -a * 1.7 (cancellation).  Inputs are chosen around the fp32 denormal range.
#include <hip/hip_runtime.h>

__global__ void pkf32_kernel(const float* a, const float* b, float* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float x = a[i], y = b[i], sm, sa;
  float pm0, pm1, pa0, pa1;
  asm volatile("v_mul_f32 %0, %1, %2" : "=v"(sm) : "v"(x), "v"(y));
  asm volatile("v_add_f32 %0, %1, %2" : "=v"(sa) : "v"(x), "v"(y));
  asm volatile("v_mov_b32 v40, %4\n v_mov_b32 v41, %4\n v_mov_b32 v42, %5\n v_mov_b32 v43, %5\n"
               "v_pk_mul_f32 v[44:45], v[40:41], v[42:43]\n v_pk_add_f32 v[46:47], v[40:41], v[42:43]\n"
               "v_mov_b32 %0, v44\n v_mov_b32 %1, v45\n v_mov_b32 %2, v46\n v_mov_b32 %3, v47"
               : "=v"(pm0), "=v"(pm1), "=v"(pa0), "=v"(pa1) : "v"(x), "v"(y) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
  const float c = -x * 1.7f;
  float sf, pf0, pf1;
  asm volatile("v_fma_f32 %0, %1, %2, %3" : "=v"(sf) : "v"(x), "v"(y), "v"(c));
  asm volatile("v_mov_b32 v40, %2\n v_mov_b32 v41, %2\n v_mov_b32 v42, %3\n v_mov_b32 v43, %3\n"
               "v_mov_b32 v44, %4\n v_mov_b32 v45, %4\n v_pk_fma_f32 v[46:47], v[40:41], v[42:43], v[44:45]\n"
               "v_mov_b32 %0, v46\n v_mov_b32 %1, v47"
               : "=v"(pf0), "=v"(pf1) : "v"(x), "v"(y), "v"(c) : "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47");
  out[6 * i] = sm;
  out[6 * i + 1] = pm0;
  out[6 * i + 2] = sa;
  out[6 * i + 3] = pa0;
  out[6 * i + 4] = sf;
  out[6 * i + 5] = pf0;
}

extern "C" int pkf32_run(const float* a, const float* b, float* out, int n, void* stream) {
  pkf32_kernel<<<(n + 255) / 256, 256, 0, (hipStream_t)stream>>>(a, b, out, n);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}
