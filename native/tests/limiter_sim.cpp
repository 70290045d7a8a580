// Many-pod study of the GPU-time limiter (profiles/r2ak): N saturating pods, each with its
// own sampler (independent jittered period, as every container's lease holder runs one),
// share a processor-sharing GPU model. Uses the shim's own accounting functions
// (ratelimit.h), so only the GPU and host models are simulated.
//
//   vgpu_limiter_sim [pods] [sample_us] [seconds] [seed] [odd_weight] [pct]
//
// odd_weight > 1 makes the GPU's arbitration unfair: odd-numbered pods progress that much
// faster than the others while both are resident (the bimodal per-pod rates measured at
// 12 pods, profiles/r2ae). pct overrides the plugin's rounded-up share.
// Prints one JSON line: each pod's throughput as a fraction of the whole GPU over the
// measured window (after 1 s of warm-up), and the slowest pod against its 1/N share.
// The model has no GPU warm-up cost and no read cost, so it isolates what the sampling
// period does to the accuracy of each pod's charge.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "vgpu/ratelimit.h"

using namespace vgpu;

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 12;
  const int sample_us = argc > 2 ? atoi(argv[2]) : 1000;
  const double seconds = argc > 3 ? atof(argv[3]) : 6.0;
  const unsigned seed = argc > 4 ? (unsigned)atoi(argv[4]) : 1;
  const double odd_weight = argc > 5 ? atof(argv[5]) : 1.0;
  const int pct = argc > 6 ? atoi(argv[6]) : (100 + n - 1) / n;  // default: the plugin's rounded-up share
  // ResNet-50-like stream: 65 µs kernels enqueued every 5 µs while the gate is open, at
  // most one step (200 kernels) ahead of the GPU.
  const int64_t step_ns = 5'000, kernel_ns = 65'000, launch_ns = 5'000, depth = 200;
  const int64_t warm_ns = 1'000'000'000, end = warm_ns + (int64_t)(seconds * 1e9);
  std::vector<DeviceState> dev(n);
  std::vector<TimeShareParams> par(n);
  std::vector<int64_t> backlog(n, 0), next_launch(n, 0), next_sample(n), last_sample(n, 0);
  std::vector<double> done(n, 0);
  std::vector<int> prev_pm(n, 0);
  std::vector<bool> opened(n, false);
  std::vector<unsigned> rng(n);
  for (int i = 0; i < n; i++) {
    par[i] = timeshare_params(pct);
    dev[i].credit_ns.store(par[i].burst_ns);
    dev[i].gate_open.store(1);
    rng[i] = seed * 7919u + (unsigned)i * 104729u + 1;
    next_sample[i] = (int64_t)(rng[i] % (unsigned)(sample_us * 1000));
  }
  for (int64_t t = 0; t < end; t += step_ns) {
    for (int i = 0; i < n; i++)
      if (t >= next_launch[i] && dev[i].gate_open.load() && backlog[i] < depth * kernel_ns) {
        backlog[i] += kernel_ns;
        next_launch[i] = t + launch_ns;
      }
    double wsum = 0;
    for (int i = 0; i < n; i++)
      if (backlog[i] > 0) wsum += (i & 1) ? odd_weight : 1.0;
    for (int i = 0; i < n; i++) {
      if (backlog[i] <= 0) continue;
      int64_t prog = std::min<int64_t>(backlog[i], (int64_t)(step_ns * ((i & 1) ? odd_weight : 1.0) / wsum));
      backlog[i] -= prog;
      if (t >= warm_ns) done[i] += (double)prog;
    }
    for (int i = 0; i < n; i++) {
      if (t < next_sample[i]) continue;
      const int64_t dt = t - last_sample[i];
      last_sample[i] = t;
      // Resident waves in proportion to each pod's arbitration weight.
      auto waves = [&](int j) { return backlog[j] > 0 ? (int64_t)(32 * ((j & 1) ? odd_weight : 1.0)) : 0; };
      int64_t mine = waves(i), total = mine;
      if (mine)
        for (int j = 0; j < n; j++)
          if (j != i) total += waves(j);
      const int pm = (int)timeshare_charge(1000, mine, total);
      const int64_t charge = timeshare_interval(dt, prev_pm[i], pm, opened[i]);
      const bool was_closed = !dev[i].gate_open.load();
      timeshare_apply(dev[i], par[i], dt, charge);
      opened[i] = was_closed && dev[i].gate_open.load();
      prev_pm[i] = pm;
      rng[i] = rng[i] * 1103515245u + 12345u;
      next_sample[i] = t + sample_us * 750 + (int64_t)((rng[i] >> 8) % (unsigned)(sample_us * 500 + 1));
    }
  }
  const double win = (double)(end - warm_ns);
  double sum = 0, lo = 1, hi = 0;
  printf("{\"pods\": %d, \"pct\": %d, \"sample_us\": %d, \"seconds\": %.1f, \"seed\": %u, \"share\": [", n, pct,
         sample_us, seconds, seed);
  for (int i = 0; i < n; i++) {
    double f = done[i] / win;
    sum += f;
    lo = std::min(lo, f);
    hi = std::max(hi, f);
    printf("%s%.4f", i ? ", " : "", f);
  }
  printf("], \"aggregate\": %.4f, \"slowest_vs_1_over_n\": %.3f, \"fastest_vs_1_over_n\": %.3f}\n", sum, lo * n,
         hi * n);
  return 0;
}
