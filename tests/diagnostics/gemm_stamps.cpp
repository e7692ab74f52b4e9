// Diagnostic (GPU box): in-kernel timeline of one mf_gemm_nt launch.  Builds gemm.hip with
// MF_GEMM_STAMPS so lane 0 of every workgroup records s_memrealtime (100 MHz) at: start, first
// K-tile landed, main loop done, epilogue done; plus its XCC id and HW_ID.  Prints the launch
// span and per-phase distributions.
//   hipcc -O3 -std=c++17 --offload-arch=gfx950 -DMF_GEMM_STAMPS -I../../federated_multi_modal_amd/csrc \
//         gemm_stamps.cpp -o gemm_stamps && ./gemm_stamps M N K epi tile [aux_out]
// aux_out 0: EPI_BIAS_GELU without the pre-activation store (the forward-only eval engine)
#define MF_GEMM_STAMPS 1
#include "../../federated_multi_modal_amd/csrc/common.hip"
#include "../../federated_multi_modal_amd/csrc/gemm.hip"

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

int main(int argc, char** argv) {
  int M = argc > 1 ? atoi(argv[1]) : 6368, N = argc > 2 ? atoi(argv[2]) : 2304, K = argc > 3 ? atoi(argv[3]) : 768;
  int epi = argc > 4 ? atoi(argv[4]) : 1, tile = argc > 5 ? atoi(argv[5]) : 1;
  int BM = 128, BN = 128;
  if (tile == 2) BN = 64;
  if (tile == 3) BM = BN = 64;
  if (tile >= 20) { BM = tile == 23 || tile == 24 ? 128 : 256; BN = (tile == 20 || tile == 23 || tile >= 27) ? 256 : 128; }
  const bool aux_out = argc > 6 ? atoi(argv[6]) != 0 : true;
  // tile 27 (persistent): one stamp row per TILE (start = its loop iteration), not per workgroup
  if (tile == 10) { BM = 160; BN = 128; }
  if (tile == 15) { BM = 96; BN = 128; }
  if (tile == 16) { BM = 160; BN = 64; }
  if (tile == 26) { BM = 96; BN = 64; }
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  _Float16 *A, *B, *C, *bias, *aux;
  hipMalloc(&A, (size_t)M * K * 2); hipMalloc(&B, (size_t)N * K * 2); hipMalloc(&C, (size_t)M * N * 2);
  hipMalloc(&bias, (size_t)N * 2); hipMalloc(&aux, (size_t)M * N * 2);
  std::vector<_Float16> h((size_t)std::max(M, N) * K);
  for (auto& x : h) x = (_Float16)((rand() / (float)RAND_MAX - 0.5f) * 0.5f);
  hipMemcpy(A, h.data(), (size_t)M * K * 2, hipMemcpyHostToDevice);
  hipMemcpy(B, h.data(), (size_t)N * K * 2, hipMemcpyHostToDevice);
  hipMemset(bias, 0, N * 2); hipMemset(aux, 0, (size_t)M * N * 2);
  unsigned long long* st;
  hipMalloc(&st, (size_t)tiles * 8 * 8);
  hipMemcpyToSymbol(HIP_SYMBOL(g_stamps), &st, sizeof(st));
  for (int rep = 0; rep < 5; ++rep) {
    hipMemset(st, 0, (size_t)tiles * 64);
    int rc = mf_gemm_nt(A, K, B, K, C, N, M, N, K, bias, aux, aux_out ? aux : nullptr, N, epi, tile, 0);
    if (rc) { printf("error %s\n", mf_last_error()); return 1; }
    hipDeviceSynchronize();
  }
  std::vector<unsigned long long> s((size_t)tiles * 8);
  hipMemcpy(s.data(), st, s.size() * 8, hipMemcpyDeviceToHost);
  unsigned long long t0 = ~0ull, t3 = 0;
  for (int b = 0; b < tiles; ++b) { t0 = std::min(t0, s[b * 8]); t3 = std::max(t3, s[b * 8 + 3]); }
  auto us = [](unsigned long long d) { return d / 100.0; };  // 100 MHz ticks -> us
  std::vector<double> pro, loop, epi_t, start, end;
  for (int b = 0; b < tiles; ++b) {
    pro.push_back(us(s[b * 8 + 1] - s[b * 8])); loop.push_back(us(s[b * 8 + 2] - s[b * 8 + 1]));
    epi_t.push_back(us(s[b * 8 + 3] - s[b * 8 + 2])); start.push_back(us(s[b * 8] - t0)); end.push_back(us(s[b * 8 + 3] - t0));
  }
  auto pr = [](const char* n, std::vector<double> v) {
    std::sort(v.begin(), v.end());
    printf("%-12s min %7.2f  p10 %7.2f  med %7.2f  p90 %7.2f  max %7.2f us\n", n, v[0], v[v.size() / 10], v[v.size() / 2],
           v[v.size() * 9 / 10], v.back());
  };
  printf("M=%d N=%d K=%d epi=%d tile=%d: %d workgroups, span %.2f us, %.0f TFLOP/s over the span\n", M, N, K, epi, tile,
         tiles, us(t3 - t0), 2.0 * M * N * K / (us(t3 - t0) * 1e6));
  pr("start", start); pr("prologue", pro); pr("main loop", loop); pr("epilogue", epi_t); pr("end", end);
  // start-time histogram (rounds)
  int hist[40] = {0};
  for (double x : start) hist[std::min(39, (int)(x / (us(t3 - t0) / 40)))]++;
  printf("start histogram (40 bins over the span):");
  for (int i = 0; i < 40; ++i) printf(" %d", hist[i]);
  printf("\n");
  return 0;
}
