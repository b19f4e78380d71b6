// Sanitizer driver for the bucket engine core (csrc/comm/engine.h) through its fake in-process
// backend (csrc/engine_cpu/fake_engine.cpp): 8 emulated ranks, overlapped cycles, every wire
// format, a fusion threshold that splits ranges, and a stalled rank the watchdog must name.
// Built and run by tools/sanitize/run_engine_sanitizers.sh under ASan+UBSan and under TSan
// (the race detector for the engine's submit thread / comm thread / watchdog thread).
#include <cmath>
#include <cstdio>
#include <cstdlib>

#include "engine_cpu/fake_engine.h"

using namespace hcb;

static int check(int world, comm::Wire w, bool avg, int64_t thr, int stall_rank, int stall_ms, double warn_s) {
  const int64_t n = 100003;
  std::vector<std::vector<float>> init(world, std::vector<float>(n));
  for (int r = 0; r < world; ++r)
    for (int64_t i = 0; i < n; ++i) init[r][i] = (float)((r + 1) * ((i % 97) - 48)) * 0.125f;
  // three overlapped cycles covering the buffer in backward order, uneven ranges
  std::vector<std::vector<int64_t>> cycles = {{70000, 30003}, {20000, 50000}, {0, 20000}};
  fake::RunConfig cfg;
  cfg.world = world;
  cfg.wire = w;
  cfg.average = avg;
  cfg.threshold_bytes = thr;
  cfg.stall_rank = stall_rank;
  cfg.stall_seq = stall_rank >= 0 ? 2 : -1;
  cfg.stall_ms = stall_ms;
  cfg.warn_s = warn_s;
  fake::RunResult res = fake::run(cfg, init, cycles);
  int bad = 0;
  for (int r = 0; r < world; ++r) {
    if (res.buckets[r].size() != res.buckets[0].size()) ++bad;
    for (size_t b = 0; b < res.buckets[r].size(); ++b) {
      const auto &x = res.buckets[r][b], &y = res.buckets[0][b];
      if (x.seq != y.seq || x.off != y.off || x.len != y.len) ++bad;
      if (thr > 0 && x.len * comm::wire_bytes(w) > thr) ++bad;
    }
    for (int64_t i = 0; i < n; ++i) {
      float exp = 0.f;
      for (int q = 0; q < world; ++q) exp += fake::wire_round(init[q][i], w);
      if (avg) exp /= (float)world;
      exp = fake::wire_round(exp, w);
      if (std::fabs(res.buffers[r][i] - exp) > 1e-6f * (1.f + std::fabs(exp))) {
        ++bad;
        break;
      }
    }
  }
  if (res.size_mismatches) ++bad;
  if (stall_rank >= 0 && warn_s > 0 && res.warnings.empty()) ++bad;
  std::printf("world=%d wire=%d avg=%d thr=%lld stall=%d: %zu buckets/rank, %zu warnings -> %s\n", world, (int)w,
              (int)avg, (long long)thr, stall_rank, res.buckets[0].size(), res.warnings.size(), bad ? "FAIL" : "ok");
  return bad;
}

int main() {
  int bad = 0;
  bad += check(8, comm::Wire::F32, false, 64 * 1024, -1, 0, 0);
  bad += check(8, comm::Wire::BF16, true, 48 * 1024, -1, 0, 0);
  bad += check(8, comm::Wire::F16, false, 0, -1, 0, 0);
  bad += check(4, comm::Wire::F32, true, 128 << 20, -1, 0, 0);
  bad += check(8, comm::Wire::F32, false, 32 * 1024, 3, 300, 0.05);
  std::printf(bad ? "ENGINE STRESS FAILED\n" : "ENGINE STRESS OK\n");
  return bad ? 1 : 0;
}
