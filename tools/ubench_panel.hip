// Dev microbenchmark: timeline of one k_chol_panel launch (N = 4096, first
// panel) from the SMG_PANEL_TRACE event log, against the same panel done by
// the per-step launches (potrf / TRSM / trapezoid update).
#define SMG_PANEL_TRACE 1
#include "../math_amd/csrc/cholesky.hip"
#include <cstdio>
#include <vector>
#include <cmath>

int main(int argc, char** argv) {
  const int nha = argc > 1 ? atoi(argv[1]) : 5;  // column helper workgroups A (tiles 3..7)
  const int nhb = argc > 2 ? atoi(argv[2]) : 4;  // and B (tiles 4..7)
  const int nh = nha + nhb;
  const int n = 4096, J = 0, K = 512;
  std::vector<double> A((size_t)n * n);
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) A[i + (size_t)j * n] = (i == j ? n : 0.0) + 1.0 / (1.0 + i + j);
  double *dL, *dD;
  int *flags, *status;
  hipMalloc(&dL, 8ull * n * n);
  hipMalloc(&dD, 8ull * n * SMG_AUX_COLS);  // the whole aux: the inverter also writes the 128 level
  hipMalloc(&flags, 4096 * 4);
  hipMalloc(&status, 4);
  hipMemset(flags, 0, 4096 * 4);
  hipMemset(status, 0, 4);
  const int T = panel_tiles(n, J, K / 64);
  const int paired = argc > 3 ? atoi(argv[3]) : 1;  // pairs of 32-row tiles below the panel per workgroup
  const int gown = paired ? K / 64 + 1 + (T - K / 64 + 1) / 2 : T + 1;
  {  // the single-workgroup diagonal kernel alone, back to back
    hipMemcpy(dL, A.data(), 8ull * n * n, hipMemcpyHostToDevice);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int w = 0; w < 2; ++w)
      hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(512), 0, 0, dL, n, 64, dD, n, status);
    hipEventRecord(e0);
    for (int w = 0; w < 20; ++w)
      hipLaunchKernelGGL(k_potrf_diag, dim3(1), dim3(512), 0, 0, dL + 64 * (w % 8) * (n + 1), n, 64,
                         dD, n, status);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    printf("k_potrf_diag alone: %.2f us per launch\n", ms * 1000 / 20);
  }
  for (int rep = 1; rep <= 3; ++rep) {
    hipMemcpy(dL, A.data(), 8ull * n * n, hipMemcpyHostToDevice);
    int zero[PANEL_MAX_GRID] = {0};
    hipMemcpyToSymbol(HIP_SYMBOL(g_panel_trace_n), zero, sizeof(zero));
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL(k_chol_panel, dim3(gown + nh), dim3(512), 0, 0, dL, n, n, J, K, dD, n, flags, rep,
                       status, gown, nha, paired);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms;
    hipEventElapsedTime(&ms, e0, e1);
    int st;
    hipMemcpy(&st, status, 4, hipMemcpyDeviceToHost);
    printf("panel kernel: %.1f us status %d\n", ms * 1000, st);
    if (rep < 3) continue;
    {  // host reference for the panel columns [0, K): left-looking Cholesky
      std::vector<double> Lh((size_t)n * K, 0.0), Lg((size_t)n * n);
      hipMemcpy(Lg.data(), dL, 8ull * n * n, hipMemcpyDeviceToHost);
      for (int j = 0; j < K; ++j) {
        double d = A[j + (size_t)j * n];
        for (int k = 0; k < j; ++k) d -= Lh[j + (size_t)k * n] * Lh[j + (size_t)k * n];
        d = sqrt(d);
        Lh[j + (size_t)j * n] = d;
        for (int i = j + 1; i < n; ++i) {
          double v = A[i + (size_t)j * n];
          for (int k = 0; k < j; ++k) v -= Lh[i + (size_t)k * n] * Lh[j + (size_t)k * n];
          Lh[i + (size_t)j * n] = v / d;
        }
      }
      for (int t = 0; t < n / 64; ++t) {
        printf("tile %2d:", t);
        for (int jb = 0; jb < K / 64; ++jb) {
          double e = 0;
          for (int c = 64 * jb; c < 64 * jb + 64; ++c)
            for (int r = 64 * t; r < 64 * t + 64; ++r)
              if (r >= c) e = fmax(e, fabs(Lh[r + (size_t)c * n] - Lg[r + (size_t)c * n]));
          printf(" %.1e", e);
        }
        printf("\n");
        if (t == 6) t = n / 64 - 3;
      }
    }
    std::vector<unsigned long long> tr(PANEL_MAX_GRID * 128);
    std::vector<int> cnt(PANEL_MAX_GRID);
    hipMemcpyFromSymbol(tr.data(), HIP_SYMBOL(g_panel_trace), tr.size() * 8);
    hipMemcpyFromSymbol(cnt.data(), HIP_SYMBOL(g_panel_trace_n), cnt.size() * 4);
    unsigned long long t0 = ~0ull;
    for (int w = 0; w < gown + nh; ++w)
      for (int k = 0; k < cnt[w] && k < 64; ++k) t0 = std::min(t0, tr[w * 128 + 2 * k]);
    for (int w : {0, 1, 6, 7, 8, 11, gown - 1, gown, gown + 4, gown + 5, gown + 8}) {
      if (w >= gown + nh) continue;
      printf("WG %d:", w);
      for (int k = 0; k < cnt[w] && k < 64; ++k) {
        const unsigned long long c = tr[w * 128 + 2 * k + 1];
        printf(" [j%llu t%llu p%llu %.2fus]", c >> 16, (c >> 8) & 255, c & 255,
               (tr[w * 128 + 2 * k] - t0) / 100.0);
      }
      printf("\n");
    }
  }
  return 0;
}
