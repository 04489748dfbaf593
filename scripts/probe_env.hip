// Diagnostic probe (not part of the library): per-phase s_memtime stamps of the ring Pong step
// kernel, per workgroup, for wave 0 and wave 1.  Stamps go to their own buffer only.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 -Icsrc scripts/probe_env.hip -o /tmp/probe_env
//   /tmp/probe_env [envs]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
__device__ unsigned long long g_stamps[8192][2][5];
#define PONG_STAMP(i)                                                                            \
  if ((threadIdx.x & 63) == 0 && threadIdx.x < 128)                                              \
    g_stamps[blockIdx.x][threadIdx.x >> 6][i] = __builtin_amdgcn_s_memtime();
__device__ unsigned long long g_loop[24][2];
#define PONG_LOOP_STAMP(it, slow)                                                                  \
  if (blockIdx.x == 0 && threadIdx.x == 0) { g_loop[it][0] = __builtin_amdgcn_s_memtime(); g_loop[it][1] = (slow); }
#include "../csrc/envs.hip"

int main(int argc, char** argv) {
  const int B = argc > 1 ? atoi(argv[1]) : 2048;
  const int NST = 12, HW = 160 * 120;
  std::vector<int> st(B * NST, 0);
  for (int b = 0; b < B; ++b) { st[b * NST + 4] = 100 * 16; st[b * NST + 5] = 100 * 16; st[b * NST + 8] = 5; }
  std::vector<int> tab(8 * 160);
  for (int y = 0; y < 160; ++y) { tab[y] = (y * 210) / 160; tab[160 + y] = std::min(209, tab[y] + 1); tab[320 + y] = 1024; tab[480 + y] = 1024; }
  for (int x = 0; x < 120; ++x) { tab[640 + x] = (x * 160) / 120; tab[800 + x] = std::min(159, tab[640 + x] + 1); tab[960 + x] = 1024; tab[1120 + x] = 1024; }
  int *dst, *dtab, *dact; unsigned *dctr; float *drew, *dep; unsigned char *ddone, *dfc, *dframes;
  hipMalloc(&dst, B * NST * 4); hipMalloc(&dtab, pong_tables_ints() * 4); hipMalloc(&dact, B * 4); hipMalloc(&dctr, B * 4);
  hipMalloc(&drew, B * 4); hipMalloc(&dep, B * 4); hipMalloc(&ddone, B); hipMalloc(&dfc, 2 * B);
  hipMalloc(&dframes, (size_t)B * HW);
  hipMemcpy(dst, st.data(), B * NST * 4, hipMemcpyHostToDevice);
  hipMemcpy(dtab, tab.data(), 8 * 160 * 4, hipMemcpyHostToDevice);
  launch_pong_digit_tables(dtab, 87, 142, 130, 150, 200, nullptr);
  hipMemset(dact, 0, B * 4); hipMemset(dctr, 0, B * 4); hipMemset(dfc, 0, 2 * B);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  for (int it = 0; it < 20; ++it)
    launch_pong_step_ring(dst, dctr, dact, 6, dframes, HW, dfc, dfc + B, dtab, drew, ddone, dep, B, 7, 4, 100000, 6,
                          87, 142, 130, 150, 200, 0, nullptr);
  hipEventRecord(a, 0);
  launch_pong_step_ring(dst, dctr, dact, 6, dframes, HW, dfc, dfc + B, dtab, drew, ddone, dep, B, 7, 4, 100000, 6, 87,
                        142, 130, 150, 200, 0, nullptr);
  hipEventRecord(b, 0);
  hipEventSynchronize(b);
  float ms; hipEventElapsedTime(&ms, a, b);
  std::vector<unsigned long long> h((size_t)8192 * 2 * 5);
  hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(g_stamps), h.size() * 8);
  unsigned long long t0 = ~0ull, t1 = 0;
  std::vector<double> d[2][4];
  for (int w = 0; w < B; ++w)
    for (int v = 0; v < 2; ++v) {
      const unsigned long long* s = &h[((size_t)w * 2 + v) * 5];
      t0 = std::min(t0, s[0]); t1 = std::max(t1, s[4]);
      for (int k = 0; k < 4; ++k) d[v][k].push_back((double)(s[k + 1] - s[k]));
    }
  printf("envs %d kernel %.1f us, stamp span %.0f cycles\n", B, ms * 1e3, (double)(t1 - t0));
  const char* nm[4] = {"prologue+physics", "barrier1", "tables+barrier2", "render loop"};
  for (int v = 0; v < 2; ++v)
    for (int k = 0; k < 4; ++k) {
      auto& x = d[v][k]; std::sort(x.begin(), x.end());
      printf("wave%d %-18s median %8.0f  p90 %8.0f cycles\n", v, nm[k], x[x.size() / 2], x[x.size() * 9 / 10]);
    }
  unsigned long long lp[24][2];
  hipMemcpyFromSymbol(lp, HIP_SYMBOL(g_loop), sizeof(lp));
  printf("wg0 wave0 per-iteration cycles (row rect mask):");
  for (int it = 1; it < 19; ++it) printf(" %llu(%llu)", lp[it][0] - lp[it - 1][0], lp[it - 1][1]);
  printf("\n");
  return 0;
}
