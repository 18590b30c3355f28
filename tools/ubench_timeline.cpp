// Dev tool: device-clock timeline of the GP step's Cholesky panels (start /
// end of every k_chol_panel launch, SMG_PANEL_TIMELINE build of
// cholesky.hip) inside whole evaluations, with stamps at the step's start and
// end -- the panel-to-panel gaps without a profiler.  Built by
// tools/build_ubench_timeline.sh; prints one evaluation's panels (us from the
// step's first stamp) and the per-eval totals.
#include "../math_amd/bench/smg_bench.cpp"
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <vector>

extern "C" int smg_dev_timeline(smg_ctx* ctx, int stamp_slot, unsigned long long* out);
extern "C" void smg_dev_timeline_host(double* out);
static double host_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int n = 4096;
  std::vector<double> x(n), y(n);
  unsigned s = 12345;
  auto u = [&] { s = s * 1103515245u + 12345u; return (s >> 8) / double(1 << 24); };
  for (int i = 0; i < n; ++i) {
    x[i] = -10 + 20 * u();
    y[i] = std::sin(x[i]) + 0.3 * (u() - 0.5);
  }
  if (smg_bench_gp_init(0, n, x.data(), y.data())) return 1;
  double th[3] = {1.0, 1.5, 0.3}, fx, g[3];
  for (int w = 0; w < 5; ++w) smg_bench_gp_step(th, &fx, g);
  std::vector<unsigned long long> tl(192);
  smg_ctx* c = stan::math::amd::ctx();
  for (int rep = 0; rep < 3; ++rep) {
    std::fill(tl.begin(), tl.end(), 0ull);
    smg_sync(c);
    const double h0 = host_us();  // (the idle device runs the stamp right away: its clock anchor)
    smg_dev_timeline(c, 0, nullptr);
    smg_bench_gp_step(th, &fx, g);
    smg_dev_timeline(c, 1, nullptr);
    smg_sync(c);
    smg_dev_timeline(c, -1, tl.data());
    const unsigned long long t0 = tl[128], t1 = tl[129];
    std::vector<double> hl(64);
    smg_dev_timeline_host(hl.data());
    std::vector<std::pair<unsigned long long, unsigned long long>> p;
    std::vector<std::pair<unsigned long long, double>> ph;  // device start, host launch (us from the anchor)
    for (int e = 0; e < 64; ++e)
      if (tl[2 * e] >= t0 && tl[2 * e] <= t1) {
        p.push_back({tl[2 * e], tl[2 * e + 1]});
        ph.push_back({tl[2 * e], hl[e] - h0});
      }
    std::sort(p.begin(), p.end());
    std::sort(ph.begin(), ph.end());
    printf("eval %d: %.1f us (stamp to stamp), %zu panels:", rep, (t1 - t0) / 100.0, p.size());
    double busy = 0;
    for (size_t k = 0; k < p.size(); ++k) {
      printf(" [%.1f-%.1f]", (p[k].first - t0) / 100.0, (p[k].second - t0) / 100.0);
      busy += (p[k].second - p[k].first) / 100.0;
    }
    printf("\n  host launch calls (us from the anchor stamp):");
    for (auto& q : ph) printf(" %.1f", q.second);
    printf("\n  panels busy %.1f us, first start %.1f, last end %.1f, end->stamp %.1f\n", busy,
           p.empty() ? 0.0 : (p[0].first - t0) / 100.0, p.empty() ? 0.0 : (p.back().second - t0) / 100.0,
           p.empty() ? 0.0 : (t1 - p.back().second) / 100.0);
  }
  return 0;
}
