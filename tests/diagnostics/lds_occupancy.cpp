// Diagnostic (GPU box): how many workgroups the dispatcher co-locates on one CU for a given LDS size and
// block size.  Each workgroup records s_memrealtime at start / end and its HW_ID (CU / SE) and spins for
// ~20 us, so every co-resident pair overlaps; the peak number of overlapping workgroups per CU is printed
// next to hipOccupancyMaxActiveBlocksPerMultiprocessor's answer.
//   hipcc -O3 --offload-arch=gfx950 lds_occupancy.cpp -o lds_occ && ./lds_occ
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <map>
#include <vector>

__global__ void spin_kernel(unsigned long long* st, int spin_ticks) {
  extern __shared__ float dyn[];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    st[blockIdx.x * 4 + 0] = t0;
    st[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_ID
    st[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));  // XCC_ID
  }
  dyn[threadIdx.x] = (float)threadIdx.x;  // touch LDS
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0) st[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime() + (unsigned long long)dyn[5];
}

// the fused text kernel's footprint: 73 728 B of static LDS, 384 threads, and (HIGH_VGPR) a VGPR count
// forced to >= 120 by clobbering v119
template <bool HIGH_VGPR>
__global__ __launch_bounds__(384) void spin_static_kernel(unsigned long long* st, int spin_ticks) {
  __shared__ float sl[73728 / 4];
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  if (threadIdx.x == 0) {
    st[blockIdx.x * 4 + 0] = t0;
    st[blockIdx.x * 4 + 2] = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));
    st[blockIdx.x * 4 + 3] = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));
  }
  if constexpr (HIGH_VGPR) asm volatile("v_mov_b32 v119, 0" ::: "v119");
  sl[threadIdx.x] = (float)threadIdx.x;
  while (__builtin_amdgcn_s_memrealtime() - t0 < (unsigned long long)spin_ticks) __builtin_amdgcn_s_sleep(2);
  __syncthreads();
  if (threadIdx.x == 0) st[blockIdx.x * 4 + 1] = __builtin_amdgcn_s_memrealtime() + (unsigned long long)sl[5];
}

static int peak_per_cu(const std::vector<unsigned long long>& h, int nblk) {
  std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;
  for (int b = 0; b < nblk; ++b) {
    const unsigned long long cu = (h[b * 4 + 3] << 32) | (h[b * 4 + 2] & 0xff00ull);
    ev[cu].push_back({h[b * 4 + 0], 1});
    ev[cu].push_back({h[b * 4 + 1], -1});
  }
  int peak = 0;
  for (auto& kv : ev) {
    auto& v = kv.second;
    std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
    int cur = 0;
    for (auto& e : v) { cur += e.second; peak = std::max(peak, cur); }
  }
  return peak;
}

int main() {
  const int nblk = 2048;
  unsigned long long* st;
  hipMalloc(&st, (size_t)nblk * 4 * 8);
  std::vector<unsigned long long> h((size_t)nblk * 4);
  const int threads[] = {256, 384, 512, 896};
  const int lds_kb[] = {16, 40, 53, 64, 72, 76, 80};
  hipFuncSetAttribute((const void*)spin_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  for (int nt : threads) {
    for (int kb : lds_kb) {
      const size_t bytes = (size_t)kb * 1024;
      int occ = 0;
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spin_kernel, nt, bytes);
      hipMemset(st, 0, (size_t)nblk * 4 * 8);
      spin_kernel<<<nblk, nt, bytes>>>(st, 2000);  // 20 us at 100 MHz
      if (hipDeviceSynchronize() != hipSuccess) { printf("launch failed nt=%d kb=%d\n", nt, kb); return 1; }
      hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
      // per (xcc, se, cu) peak overlap
      std::map<unsigned long long, std::vector<std::pair<unsigned long long, int>>> ev;
      for (int b = 0; b < nblk; ++b) {
        const unsigned long long hw = h[b * 4 + 2], xcc = h[b * 4 + 3];
        const unsigned long long cu = (xcc << 32) | (hw & 0xff00ull) | ((hw >> 13) & 0x7ull);  // SE, SH, CU id bits
        ev[cu].push_back({h[b * 4 + 0], 1});
        ev[cu].push_back({h[b * 4 + 1], -1});
      }
      int peak = 0;
      for (auto& kv : ev) {
        auto& v = kv.second;
        std::sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.first != b.first ? a.first < b.first : a.second < b.second; });
        int cur = 0;
        for (auto& e : v) { cur += e.second; peak = std::max(peak, cur); }
      }
      printf("threads %4d LDS %3d KB: occupancy API %d per CU, measured peak %d per CU (%zu CUs seen)\n", nt, kb, occ,
             peak, ev.size());
    }
  }
  for (int hv = 0; hv < 2; ++hv) {
    int occ = 0;
    if (hv) hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spin_static_kernel<true>, 384, 0);
    else hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, spin_static_kernel<false>, 384, 0);
    hipMemset(st, 0, (size_t)nblk * 4 * 8);
    if (hv) spin_static_kernel<true><<<nblk, 384>>>(st, 2000);
    else spin_static_kernel<false><<<nblk, 384>>>(st, 2000);
    if (hipDeviceSynchronize() != hipSuccess) { printf("static launch failed\n"); return 1; }
    hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost);
    printf("static 72 KB LDS, 384 threads, %s VGPRs: occupancy API %d per CU, measured peak %d per CU\n",
           hv ? ">= 120" : "few", occ, peak_per_cu(h, nblk));
  }
  return 0;
}
