// Diagnostic (GPU box): in-kernel timeline of the fused in-projection + attention forward
// (qkv_attn_fwd_kernel).  Builds attention.hip with MF_ATTN_STAMPS: lane 0 of every workgroup records
// s_memrealtime (100 MHz) at the start, after the GEMM phase, after the q/k/v images are written, at the end.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 qkv_stamps.cpp -o qkv_stamps && ./qkv_stamps N L H causal
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
  _Float16 *x, *w, *b, *qkv, *o;
  float* lse;
  hipMalloc(&x, (size_t)R * D * 2); hipMalloc(&w, (size_t)3 * D * D * 2); hipMalloc(&b, (size_t)3 * D * 2);
  hipMalloc(&qkv, (size_t)R * 3 * D * 2); hipMalloc(&o, (size_t)R * D * 2); hipMalloc(&lse, (size_t)NH * L * 4);
  std::vector<_Float16> h((size_t)R * D);
  for (auto& v : h) v = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 2.f);
  hipMemcpy(x, h.data(), (size_t)R * D * 2, hipMemcpyHostToDevice);
  std::vector<_Float16> hw((size_t)3 * D * D);
  for (auto& v : hw) v = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.07f);
  hipMemcpy(w, hw.data(), hw.size() * 2, hipMemcpyHostToDevice);
  hipMemset(b, 0, (size_t)3 * D * 2);
  {
    int nb = 0;
    if (D == 768)
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, qkv_attn_fwd_vision_kernel, 896, 0);
    else
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, qkv_attn_fwd_text_kernel, 384, 0);
    printf("occupancy API: %d workgroups per CU\n", nb);
  }
  unsigned long long* st;
  const size_t nst = (size_t)NH * 8;
  hipMalloc(&st, nst * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_astamps), &st, sizeof(st));
  for (int rep = 0; rep < 6; ++rep) {
    hipMemset(st, 0, nst * 8);
    int rc = mf_qkv_attention_fwd(x, D, R, w, b, qkv, 3 * D, o, D, lse, L, N, L, H, causal, 0);
    if (rc) { printf("error %s\n", mf_last_error()); return 1; }
    hipDeviceSynchronize();
  }
  std::vector<unsigned long long> s(nst);
  hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, t3 = 0;
  for (int g = 0; g < NH; ++g) { t0 = std::min(t0, s[g * 8]); t3 = std::max(t3, s[g * 8 + 3]); }
  printf("qkv_attn N=%d L=%d H=%d causal=%d: %d workgroups, span %.2f us\n", N, L, H, causal, NH, (t3 - t0) / 100.0);
  const char* fn[3] = {"gemm", "images", "attn+store"};
  for (int k = 0; k < 3; ++k) {
    std::vector<double> v;
    for (int g = 0; g < NH; ++g) v.push_back((s[g * 8 + k + 1] - s[g * 8 + k]) / 100.0);
    std::sort(v.begin(), v.end());
    printf("  %-10s min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", fn[k], v[0], v[v.size() / 2], v[v.size() * 9 / 10], v.back());
  }
  std::vector<double> st0, en;
  for (int g = 0; g < NH; ++g) { st0.push_back((s[g * 8] - t0) / 100.0); en.push_back((s[g * 8 + 3] - t0) / 100.0); }
  std::sort(st0.begin(), st0.end()); std::sort(en.begin(), en.end());
  printf("  start      min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", st0[0], st0[st0.size() / 2], st0[st0.size() * 9 / 10], st0.back());
  printf("  end        min %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", en[0], en[en.size() / 2], en[en.size() * 9 / 10], en.back());
  // peak number of workgroups resident at once (start/end sweep): 256 x workgroups-per-CU when the grid is large
  std::vector<std::pair<unsigned long long, int>> ev;
  for (int g = 0; g < NH; ++g) { ev.push_back({s[g * 8], 1}); ev.push_back({s[g * 8 + 3], -1}); }
  std::sort(ev.begin(), ev.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
  int cur = 0, peak = 0;
  for (auto& e : ev) { cur += e.second; peak = std::max(peak, cur); }
  printf("  peak resident workgroups %d\n", peak);
  return 0;
}
