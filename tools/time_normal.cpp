// Config-1 latency breakdown (one gradient of normal_lpdf(theta | 0, 1),
// N = 1024 host vars): host tape alone, the fused device call alone, the
// whole gradient.  g++ -O2 -std=c++17 -Imath_amd/include -Iinclude -isystem <eigen>
//   tools/time_normal.cpp -Lmath_amd/lib -lsmg_hip -Wl,-rpath,<abs>/math_amd/lib
#include <stan/math.hpp>

#include <chrono>
#include <cstdio>

using namespace stan::math;

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const int N = 1024, reps = 20000;
  std::vector<double> th(N), g;
  for (int i = 0; i < N; ++i) th[i] = 0.001 * (i - 512);
  double fx = 0;
  auto f_normal = [](const std::vector<var>& t) { return normal_lpdf(t, 0.0, 1.0); };
  auto f_host = [](const std::vector<var>& t) { return t[0] * 2.0; };
  for (int r = 0; r < 200; ++r) gradient(f_normal, th, fx, g);
  double t0 = now();
  for (int r = 0; r < reps; ++r) gradient(f_host, th, fx, g);
  const double t_host = (now() - t0) / reps;
  smg_ctx* c = amd::ctx();
  double* st = static_cast<double*>(smg_pinned_io(c, (8 + 2 * N + 2) * sizeof(double)));
  for (int i = 0; i < N; ++i) st[8 + i] = th[i];
  st[8 + N] = 0.0;
  st[9 + N] = 1.0;
  t0 = now();
  for (int r = 0; r < reps; ++r)
    smg_normal_lpdf_fused(c, st + 8, nullptr, nullptr, 0.0, 0.0, 1.0, N, 7, st, st + 10 + N, nullptr, nullptr);
  const double t_fused = (now() - t0) / reps;
  t0 = now();
  for (int r = 0; r < reps; ++r) gradient(f_normal, th, fx, g);
  const double t_grad = (now() - t0) / reps;
  std::printf("{\"host_tape_us\": %.2f, \"fused_call_us\": %.2f, \"gradient_us\": %.2f, \"fx\": %.12g}\n",
              t_host * 1e6, t_fused * 1e6, t_grad * 1e6, fx);
  return 0;
}
