// pybind11 bindings for the mihvd host runtime (module mihvd._native._mihvd_runtime).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "control.h"
#include "runtime.h"

namespace py = pybind11;
using namespace mihvd;

PYBIND11_MODULE(_mihvd_runtime, m) {
  m.doc() = "mihvd native host runtime: bucket planner, controller, timeline, stall inspector, "
            "TCP key-value store, collective negotiation engine";

  py::class_<TensorSpec>(m, "TensorSpec")
      .def(py::init<>())
      .def(py::init([](int64_t numel, int elem_size, int dtype, int device) {
             TensorSpec s;
             s.numel = numel;
             s.elem_size = elem_size;
             s.dtype = dtype;
             s.device = device;
             return s;
           }),
           py::arg("numel"), py::arg("elem_size"), py::arg("dtype") = 0, py::arg("device") = 0)
      .def_readwrite("numel", &TensorSpec::numel)
      .def_readwrite("elem_size", &TensorSpec::elem_size)
      .def_readwrite("dtype", &TensorSpec::dtype)
      .def_readwrite("device", &TensorSpec::device);

  py::class_<BucketPlan>(m, "BucketPlan")
      .def_readonly("members", &BucketPlan::members)
      .def_readonly("offsets", &BucketPlan::offsets)
      .def_readonly("numel", &BucketPlan::numel)
      .def_readonly("dtype", &BucketPlan::dtype)
      .def_readonly("device", &BucketPlan::device)
      .def_readonly("tensor_bucket", &BucketPlan::tensor_bucket)
      .def_readonly("tensor_offset", &BucketPlan::tensor_offset)
      .def("__len__", [](const BucketPlan& p) { return p.members.size(); });

  m.def("plan_buckets", &plan_buckets, py::arg("specs"), py::arg("order"),
        py::arg("threshold_bytes"), py::arg("align_bytes") = 256);

  py::class_<Controller>(m, "Controller")
      .def(py::init<std::vector<int>, int, int>(), py::arg("tensor_bucket"),
           py::arg("num_buckets"), py::arg("passes_per_step") = 1)
      .def("mark_ready", &Controller::mark_ready)
      .def("flush", &Controller::flush)
      .def("reset", &Controller::reset)
      .def("pending_in_bucket", &Controller::pending_in_bucket)
      .def_property_readonly("launched", &Controller::launched)
      .def_property_readonly("num_buckets", &Controller::num_buckets)
      .def_property_readonly("passes_per_step", &Controller::passes_per_step);

  m.def("fnv1a64", [](const std::string& s) { return fnv1a64(s); });
  m.def("tensor_signature", &tensor_signature);

  py::class_<Timeline>(m, "Timeline")
      .def(py::init<const std::string&, int>(), py::arg("path"), py::arg("rank") = 0)
      .def("begin", &Timeline::begin, py::arg("name"), py::arg("cat") = "op", py::arg("tid") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("end", &Timeline::end, py::arg("name"), py::arg("cat") = "op", py::arg("tid") = 0,
           py::call_guard<py::gil_scoped_release>())
      .def("complete", &Timeline::complete, py::arg("name"), py::arg("cat"), py::arg("tid"),
           py::arg("ts_us"), py::arg("dur_us"))
      .def("instant", &Timeline::instant, py::arg("name"), py::arg("cat") = "op",
           py::arg("tid") = 0)
      .def("counter", &Timeline::counter)
      .def("now_us", &Timeline::now_us)
      .def("flush", &Timeline::flush, py::call_guard<py::gil_scoped_release>())
      .def("close", &Timeline::close, py::call_guard<py::gil_scoped_release>())
      .def_property_readonly("events_written", &Timeline::events_written)
      .def_property_readonly("path", &Timeline::path);

  py::class_<StallReport>(m, "StallReport")
      .def_readonly("name", &StallReport::name)
      .def_readonly("age_s", &StallReport::age_s);

  py::class_<StallInspector>(m, "StallInspector")
      .def(py::init<double, double, double, int>(), py::arg("warn_s") = 60.0,
           py::arg("shutdown_s") = 0.0, py::arg("poll_s") = 1.0, py::arg("rank") = 0)
      .def("submit", &StallInspector::submit)
      .def("complete", &StallInspector::complete)
      .def("outstanding", &StallInspector::outstanding, py::arg("older_than_s") = 0.0)
      .def("num_outstanding", &StallInspector::num_outstanding)
      .def("start", &StallInspector::start)
      .def("stop", &StallInspector::stop, py::call_guard<py::gil_scoped_release>())
      .def("set_hard_abort", &StallInspector::set_hard_abort)
      .def_property_readonly("stalled", &StallInspector::stalled)
      .def_property_readonly("warnings_emitted", &StallInspector::warnings_emitted);

  py::class_<FaultAction>(m, "FaultAction")
      .def_readonly("kind", &FaultAction::kind)
      .def_readonly("rank", &FaultAction::rank)
      .def_readonly("step", &FaultAction::step)
      .def_readonly("args", &FaultAction::args);

  py::class_<FaultPlan>(m, "FaultPlan")
      .def(py::init<const std::string&>())
      .def("due", &FaultPlan::due)
      .def_property_readonly("actions", &FaultPlan::actions);

  py::class_<HealthMonitor>(m, "HealthMonitor")
      .def(py::init<int, double, int>(), py::arg("rank") = 0, py::arg("poll_s") = 0.5, py::arg("exit_code") = 134)
      .def("attach_rccl", &HealthMonitor::attach_rccl, py::arg("comm"), py::arg("lib_path"))
      .def("detach_rccl", &HealthMonitor::detach_rccl, py::arg("comm"))
      .def("inject_error", &HealthMonitor::inject_error, py::arg("code"), py::arg("what") = "test")
      .def("watch_word", &HealthMonitor::watch_word, py::arg("addr"), py::arg("label"))
      .def("unwatch_word", &HealthMonitor::unwatch_word, py::arg("addr"))
      .def_property_readonly("num_words", &HealthMonitor::num_words)
      .def("poll_once", [](HealthMonitor& h) {
             std::string what;
             int e;
             {
               py::gil_scoped_release nogil;
               e = h.poll_once(&what);
             }
             return py::make_tuple(e, what);
           })
      .def("start", &HealthMonitor::start)
      .def("stop", &HealthMonitor::stop, py::call_guard<py::gil_scoped_release>())
      .def("set_abort_process", &HealthMonitor::set_abort_process)
      .def_property_readonly("error", &HealthMonitor::error)
      .def_property_readonly("polls", &HealthMonitor::polls)
      .def_property_readonly("num_comms", &HealthMonitor::num_comms);

  py::class_<StepStats>(m, "StepStats")
      .def(py::init<size_t>(), py::arg("window") = 100)
      .def("add", &StepStats::add)
      .def("mean", &StepStats::mean)
      .def("percentile", &StepStats::percentile)
      .def("reset", &StepStats::reset)
      .def_property_readonly("count", &StepStats::count);

  // ---- control plane: key-value store + negotiation engine (control.h) ----
  using gil_release = py::call_guard<py::gil_scoped_release>;
  py::class_<StoreServer>(m, "StoreServer")
      .def(py::init<const std::string&, int>(), py::arg("host") = "0.0.0.0", py::arg("port") = 0)
      .def_property_readonly("port", &StoreServer::port)
      .def_property_readonly("num_connections", &StoreServer::num_connections)
      .def("num_keys", &StoreServer::num_keys)
      .def("stop", &StoreServer::stop, gil_release());

  py::class_<EngineNegotiation>(m, "EngineNegotiation")
      .def(py::init<const std::string&, int, int, int, const std::string&, int, int>(), py::arg("host"),
           py::arg("port"), py::arg("rank"), py::arg("world"), py::arg("prefix"), py::arg("cap") = 256,
           py::arg("announce_k") = 64, gil_release())
      .def("want", &EngineNegotiation::want)
      .def("slot", &EngineNegotiation::slot)
      .def("num_slots", &EngineNegotiation::num_slots)
      .def("negotiate", &EngineNegotiation::negotiate, py::arg("pending"), py::arg("stop") = false, gil_release())
      .def("announce_round", &EngineNegotiation::announce_round, gil_release())
      .def("plan", [](const EngineNegotiation& e, const std::vector<int32_t>& summed, const std::vector<int64_t>& bytes,
                      const std::vector<int64_t>& key, int64_t threshold) {
             std::vector<int> partial;
             auto groups = e.plan(summed, bytes, key, threshold, &partial);
             return py::make_tuple(groups, partial);
           })
      .def_property_readonly("announces", &EngineNegotiation::announces)
      .def_property_readonly("max_fresh", &EngineNegotiation::max_fresh)
      .def_property_readonly("rounds", &EngineNegotiation::rounds);
  m.def("engine_signature_hash", [](const std::string& sig) { return (int64_t)engine_fnv32(sig); });

  py::class_<StoreClient>(m, "StoreClient")
      .def(py::init<const std::string&, int, double>(), py::arg("host"), py::arg("port"),
           py::arg("connect_timeout_s") = 60.0, gil_release())
      .def("set", [](StoreClient& c, const std::string& k, const std::string& v) {
             py::gil_scoped_release nogil;
             c.set(k, v);
           })
      .def("get", [](StoreClient& c, const std::string& k, double timeout_s) {
             std::string v;
             {
               py::gil_scoped_release nogil;
               v = c.get(k, timeout_s);
             }
             return py::bytes(v);
           }, py::arg("key"), py::arg("timeout_s") = -1.0)
      .def("try_get", [](StoreClient& c, const std::string& k, double timeout_s) -> py::object {
             std::string v;
             bool ok;
             {
               py::gil_scoped_release nogil;
               ok = c.try_get(k, timeout_s, &v);
             }
             if (!ok) return py::none();
             return py::bytes(v);
           }, py::arg("key"), py::arg("timeout_s") = 0.0)
      .def("add", &StoreClient::add, gil_release())
      .def("check", &StoreClient::check, gil_release())
      .def("wait", &StoreClient::wait, py::arg("keys"), py::arg("timeout_s") = -1.0, gil_release())
      .def("compare_set", [](StoreClient& c, const std::string& k, const std::string& e, const std::string& d) {
             std::string v;
             {
               py::gil_scoped_release nogil;
               v = c.compare_set(k, e, d);
             }
             return py::bytes(v);
           })
      .def("delete", &StoreClient::del, gil_release())
      .def("append", [](StoreClient& c, const std::string& k, const std::string& v) {
             py::gil_scoped_release nogil;
             c.append(k, v);
           })
      .def("num_keys", &StoreClient::num_keys, gil_release())
      .def("close", &StoreClient::close, gil_release())
      .def_property_readonly("host", &StoreClient::host)
      .def_property_readonly("port", &StoreClient::port);

  py::class_<Response>(m, "NegotiationResponse")
      .def_readonly("name", &Response::name)
      .def_readonly("generation", &Response::generation)
      .def_readonly("error", &Response::error)
      .def_readonly("batch", &Response::batch);

  py::class_<StallEntry>(m, "StallEntry")
      .def_readonly("name", &StallEntry::name)
      .def_readonly("generation", &StallEntry::generation)
      .def_readonly("age_s", &StallEntry::age_s)
      .def_readonly("ready_ranks", &StallEntry::ready_ranks)
      .def_readonly("missing_ranks", &StallEntry::missing_ranks);

  py::class_<Negotiator>(m, "Negotiator")
      .def(py::init<const std::string&, int, int, int, const std::string&, double, double, double>(),
           py::arg("host"), py::arg("port"), py::arg("rank"), py::arg("size"), py::arg("prefix") = "mihvd/neg",
           py::arg("cycle_s") = 0.005, py::arg("warn_s") = 60.0, py::arg("shutdown_s") = 0.0, gil_release())
      .def("submit", &Negotiator::submit, gil_release())
      .def("poll", &Negotiator::poll, gil_release())
      .def("wait", &Negotiator::wait, py::arg("timeout_s") = -1.0, gil_release())
      .def("stalled", &Negotiator::stalled, py::arg("older_than_s") = 0.0, gil_release())
      .def("stop", &Negotiator::stop, gil_release())
      .def_property_readonly("submitted", &Negotiator::submitted)
      .def_property_readonly("responses", &Negotiator::responses)
      .def_property_readonly("warnings", &Negotiator::warnings)
      .def_property_readonly("cache_hits", &Negotiator::cache_hits)
      .def_property_readonly("records_posted", &Negotiator::records_posted);
}
