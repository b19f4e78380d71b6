// pybind11 face of the fake bucket-engine backend (CPU only; no torch, no HIP).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "fake_engine.h"

namespace py = pybind11;
using namespace hcb;

static py::dict run_py(int world, const std::vector<std::vector<float>>& init,
                       const std::vector<std::vector<int64_t>>& cycles, int wire, bool average, int64_t threshold_bytes,
                       int stall_rank, int64_t stall_seq, int stall_ms, double warn_s, int replay_steps,
                       bool heartbeat, int stall_step) {
  if (world < 1 || (int)init.size() != world) throw std::invalid_argument("init must hold one buffer per rank");
  if (wire < 0 || wire > 2) throw std::invalid_argument("wire: 0 fp32, 1 bf16, 2 fp16");
  fake::RunConfig cfg;
  cfg.world = world;
  cfg.wire = (comm::Wire)wire;
  cfg.average = average;
  cfg.threshold_bytes = threshold_bytes;
  cfg.stall_rank = stall_rank;
  cfg.stall_seq = stall_seq;
  cfg.stall_ms = stall_ms;
  cfg.warn_s = warn_s;
  cfg.replay_steps = replay_steps;
  cfg.heartbeat = heartbeat;
  cfg.stall_step = stall_step;
  fake::RunResult r;
  {
    py::gil_scoped_release nogil;
    r = fake::run(cfg, init, cycles);
  }
  py::dict out;
  out["buffers"] = r.buffers;
  py::list bks;
  for (auto& rb : r.buckets) {
    py::list l;
    for (auto& b : rb) l.append(py::make_tuple(b.seq, b.off, b.len));
    bks.append(l);
  }
  out["buckets"] = bks;
  py::list ws;
  for (auto& w : r.warnings) ws.append(py::make_tuple(w.rank, w.cycle, w.last_seq, w.waited_s));
  out["warnings"] = ws;
  out["cycles"] = r.cycles;
  out["size_mismatches"] = r.size_mismatches;
  return out;
}

static std::vector<std::tuple<int64_t, int64_t>> plan_py(const std::vector<int64_t>& ranges, int64_t threshold_bytes,
                                                         int wire) {
  auto bs = comm::plan_buckets(ranges.data(), (int64_t)ranges.size() / 2,
                               comm::bucket_elems_for(threshold_bytes, (comm::Wire)wire));
  std::vector<std::tuple<int64_t, int64_t>> out;
  for (auto& b : bs) out.emplace_back(b.off, b.len);
  return out;
}

static py::list stall_decisions(double warn_s, double abort_s, const std::vector<std::tuple<double, int, int>>& script) {
  // script: (t_seconds, enqueued_cycles, completed_cycles) -> the StallWatch action at each t
  comm::StallWatch w(warn_s, abort_s);
  const auto t0 = comm::StallWatch::clock::now();
  int enq = 0;
  py::list out;
  for (auto& [t, e, d] : script) {
    while (enq < e) w.enqueue(enq++);
    w.complete(d);
    auto now = t0 + std::chrono::duration_cast<comm::StallWatch::clock::duration>(std::chrono::duration<double>(t));
    out.append((int)w.evaluate(now));
  }
  return out;
}

PYBIND11_MODULE(_hcb_engine_cpu, m) {
  m.doc() = "CPU fake backend of the hcb gradient bucket engine (tests)";
  m.def("run", &run_py, py::arg("world"), py::arg("init"), py::arg("cycles"), py::arg("wire") = 0,
        py::arg("average") = false, py::arg("threshold_bytes") = 128ll << 20, py::arg("stall_rank") = -1,
        py::arg("stall_seq") = -1, py::arg("stall_ms") = 0, py::arg("warn_s") = 0.0, py::arg("replay_steps") = 0,
        py::arg("heartbeat") = true, py::arg("stall_step") = -1);
  m.def("plan", &plan_py, py::arg("ranges"), py::arg("threshold_bytes"), py::arg("wire") = 0);
  m.def("stall_decisions", &stall_decisions);
  m.def("f32_to_f16_bits", &fake::f32_to_f16);
  m.def("f32_to_bf16_bits", &fake::f32_to_bf16);
}
