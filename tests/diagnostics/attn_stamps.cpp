// Diagnostic (GPU box): in-kernel timeline of the fused attention backward.  Builds attention.hip
// with MF_ATTN_STAMPS: lane 0 of every workgroup records s_memrealtime (100 MHz) at kernel start,
// Q/dO staged + D/LSE ready, phase 1 (dK, dV) done, K restaged, end.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 attn_stamps.cpp -o attn_stamps && ./attn_stamps N L H causal
#define MF_ATTN_STAMPS 1
#include "../../federated_multi_modal_amd/csrc/common.hip"
#include "../../federated_multi_modal_amd/csrc/attention.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  int N = argc > 1 ? atoi(argv[1]) : 32, L = argc > 2 ? atoi(argv[2]) : 199, H = argc > 3 ? atoi(argv[3]) : 12;
  int causal = argc > 4 ? atoi(argv[4]) : 0;
  const int D = H * 64, R = N * L, NH = N * H;
  _Float16 *qkv, *o, *dout, *dqkv;
  float *lse, *ws;
  hipMalloc(&qkv, (size_t)R * 3 * D * 2); hipMalloc(&o, (size_t)R * D * 2); hipMalloc(&dout, (size_t)R * D * 2);
  hipMalloc(&dqkv, (size_t)R * 3 * D * 2); hipMalloc(&lse, (size_t)NH * L * 4); hipMalloc(&ws, (size_t)NH * L * 4);
  std::vector<_Float16> h((size_t)R * 3 * D);
  for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 2.f);
  hipMemcpy(qkv, h.data(), (size_t)R * 3 * D * 2, hipMemcpyHostToDevice);
  hipMemcpy(dout, h.data(), (size_t)R * D * 2, hipMemcpyHostToDevice);
  unsigned long long* st;
  const size_t nst = std::max<size_t>((size_t)NH * 64, 256 * 16 * 8);
  hipMalloc(&st, nst * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_astamps), &st, sizeof(st));
  const bool fwd = getenv("STAMP_FWD") != nullptr;  // time the forward (attn_fwd_kernel) instead
  mf_attention_fwd(qkv, 3 * D, o, D, lse, L, N, L, H, causal, 0);
  for (int rep = 0; rep < 5 && fwd; ++rep) {
    hipMemset(st, 0, nst * 8);
    mf_attention_fwd(qkv, 3 * D, o, D, lse, L, N, L, H, causal, 0);
    hipDeviceSynchronize();
  }
  for (int rep = 0; rep < 5 && !fwd; ++rep) {
    hipMemset(st, 0, nst * 8);
    int rc = mf_attention_bwd(qkv, 3 * D, o, D, dout, D, lse, ws, L, dqkv, 3 * D, N, L, H, causal, 0);
    if (rc) { printf("error %s\n", mf_last_error()); return 1; }
    hipDeviceSynchronize();
  }
  if (fwd) {  // output checksum (bit patterns of O, LSE): variants that claim bit-identity print the same numbers
    std::vector<short> ho((size_t)R * D);
    std::vector<float> hl((size_t)NH * L);
    hipMemcpy(ho.data(), o, ho.size() * 2, hipMemcpyDeviceToHost);
    hipMemcpy(hl.data(), lse, hl.size() * 4, hipMemcpyDeviceToHost);
    long long co = 0;
    double cl = 0;
    for (short v : ho) co += v;
    for (float v : hl) cl += v;
    printf("checksum O %lld LSE %.9g\n", co, cl);
  }
  if (fwd && getenv("STAMP_FWD4")) {  // attn_fwd4_kernel: every workgroup, id = x * qsplit + y
    const int qs = atoi(getenv("STAMP_FWD4"));
    const int nwg = NH * qs;
    std::vector<unsigned long long> s((size_t)nwg * 8);
    hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
    unsigned long long t0 = ~0ull, t3 = 0;
    for (int b = 0; b < nwg; ++b) { t0 = std::min(t0, s[b * 8]); t3 = std::max(t3, s[b * 8 + 3]); }
    printf("fwd4 N=%d L=%d H=%d: %d workgroups, span %.2f us\n", N, L, H, nwg, (t3 - t0) / 100.0);
    const char* fn[3] = {"stage K", "tile 1", "rest"};
    for (int k = 0; k < 3; ++k) {
      std::vector<double> v;
      for (int b = 0; b < nwg; ++b) v.push_back((s[b * 8 + k + 1] - s[b * 8 + k]) / 100.0);
      std::sort(v.begin(), v.end());
      printf("  %-8s min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", fn[k], v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
    }
    std::vector<double> st0, en;
    for (int b = 0; b < nwg; ++b) { st0.push_back((s[b * 8] - t0) / 100.0); en.push_back((s[b * 8 + 3] - t0) / 100.0); }
    std::sort(st0.begin(), st0.end()); std::sort(en.begin(), en.end());
    printf("  start    min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", st0[0], st0[st0.size() / 2], st0[st0.size() * 9 / 10], st0.back());
    printf("  end      min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", en[0], en[en.size() / 2], en[en.size() * 9 / 10], en.back());
    return 0;
  }
  if (fwd) {  // attn_fwd_kernel: grid (N*H, qsplit); only blockIdx.y == 0 records (its block id = x)
    std::vector<unsigned long long> s((size_t)NH * 8);
    hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
    const char* fn[3] = {"stage", "pass1(max)", "pass2(PV)"};
    for (int k = 0; k < 3; ++k) {
      std::vector<double> v;
      for (int b = 0; b < NH; ++b) if (s[b * 8 + k + 1] && s[b * 8 + k]) v.push_back((s[b * 8 + k + 1] - s[b * 8 + k]) / 100.0);
      std::sort(v.begin(), v.end());
      if (!v.empty()) printf("  fwd %-10s min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", fn[k], v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
    }
    return 0;
  }
  // backward: the fused kernel (one workgroup per head) or, with STAMP_SPLIT=s, attn_bwd_split_kernel
  // (MAPFED_ATTN_BWD=3 MAPFED_ATTN_BWD_SPLIT=s: s workgroups per head, id = head * s + split)
  const int nwg = NH * (getenv("STAMP_SPLIT") ? atoi(getenv("STAMP_SPLIT")) : 1);
  std::vector<unsigned long long> s((size_t)nwg * 8);
  hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, t4 = 0;
  for (int b = 0; b < nwg; ++b) { t0 = std::min(t0, s[b * 8]); t4 = std::max(t4, s[b * 8 + 4]); }
  auto us = [](unsigned long long d) { return d / 100.0; };
  const char* names[4] = {"stage+D", "phase1", "restage K", "phase2"};
  printf("N=%d L=%d H=%d causal=%d: %d workgroups, span %.2f us\n", N, L, H, causal, nwg, us(t4 - t0));
  for (int k = 0; k < 4; ++k) {
    std::vector<double> v;
    for (int b = 0; b < nwg; ++b) v.push_back(us(s[b * 8 + k + 1] - s[b * 8 + k]));
    std::sort(v.begin(), v.end());
    printf("  %-10s min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", names[k], v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
  }
  std::vector<double> st0, en, life;
  for (int b = 0; b < nwg; ++b) {
    st0.push_back(us(s[b * 8] - t0)); en.push_back(us(s[b * 8 + 4] - t0)); life.push_back(us(s[b * 8 + 4] - s[b * 8]));
  }
  std::sort(st0.begin(), st0.end()); std::sort(en.begin(), en.end()); std::sort(life.begin(), life.end());
  printf("  start      min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", st0[0], st0[st0.size() / 2], st0[st0.size() * 9 / 10], st0.back());
  printf("  end        min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", en[0], en[en.size() / 2], en[en.size() * 9 / 10], en.back());
  printf("  lifetime   min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", life[0], life[life.size() / 2], life[life.size() * 9 / 10], life.back());
  return 0;
}
