// Shared-memory request/response channel between actor env workers and the per-GPU inference server
// (SURVEY §2.2/§5.2).  The reference hands observations to its GPU loop through shared-memory tensors
// and an unsynchronised float "signal" polled with sleep(0.01) (agent.py:366,380-385; actor.py:268-299):
// racy by construction and ~10 ms of added latency per step.  Here:
//
//   * one POSIX shm segment: header | slot headers | per-slot request and response regions
//     (page aligned, so the server may register them as pinned host memory for direct DMA);
//   * each slot is single-producer/single-consumer with a sequence-number protocol:
//       client: write request bytes -> req_len -> req_seq.store(s+1, release) -> doorbell++ -> futex wake
//       server: observes req_seq != served (acquire), reads the request IN PLACE (zero copy), writes the
//               response -> resp_len -> resp_seq.store(req_seq, release) -> futex wake on resp_seq
//   * blocking uses Linux futexes on the shared words (no polling, no sleeps); waits drop the GIL;
//   * the server detects a dead client through the pid stored in its slot.
//
// Host-only C++ (no HIP): built as applestar_amd/_host*.so; the TSan/ASan variants of the host build
// cover this file (APPLESTAR_HOST_SANITIZE).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "shm_core.h"

namespace py = pybind11;
using namespace as_host;

namespace {

size_t buffer_bytes(const py::buffer_info& info) { return static_cast<size_t>(info.size * info.itemsize); }

class ShmServer {
 public:
  ShmServer(const std::string& name, uint32_t n_slots, uint64_t slot_bytes) : core_(name, n_slots, slot_bytes) {}
  std::vector<uint32_t> wait(int timeout_ms) {
    py::gil_scoped_release nogil;
    return core_.wait(timeout_ms);
  }
  std::vector<uint32_t> pending() { return core_.pending(); }
  py::memoryview request(uint32_t i) {
    check(i);
    if (!core_.has_request(i)) throw std::runtime_error("no pending request");
    return py::memoryview::from_memory(const_cast<char*>(core_.request_data(i)),
                                       static_cast<py::ssize_t>(core_.request_len(i)), true);
  }
  uint32_t tag(uint32_t i) { check(i); return core_.tag(i); }
  void respond(uint32_t i, py::buffer data) {
    check(i);
    py::buffer_info info = data.request();
    core_.respond(i, info.ptr, buffer_bytes(info));
  }
  std::vector<uint32_t> dead_slots() { return core_.dead_slots(); }
  void close() { core_.close(); }
  std::string name() const { return core_.segment().name(); }
  uint32_t n_slots() const { return core_.segment().n_slots(); }
  uint64_t slot_bytes() const { return core_.segment().slot_bytes(); }
  uintptr_t base_address() const { return reinterpret_cast<uintptr_t>(core_.segment().base()); }
  size_t size() const { return core_.segment().size(); }

 private:
  void check(uint32_t i) const {
    if (i >= core_.segment().n_slots()) throw std::out_of_range("slot index");
  }
  ServerCore core_;
};

class ShmClient {
 public:
  ShmClient(const std::string& name, uint32_t slot, uint32_t tag) : core_(name, slot, tag) {}
  py::bytes request(py::buffer data, int timeout_ms) {
    py::buffer_info info = data.request();
    Wait w;
    {
      py::gil_scoped_release nogil;
      w = core_.request(info.ptr, buffer_bytes(info), timeout_ms);
    }
    if (w == Wait::kClosed) throw std::runtime_error("inference server closed the channel");
    if (w == Wait::kTimeout) throw std::runtime_error("timed out waiting for the inference server");
    return py::bytes(core_.response_data(), core_.response_len());
  }
  uint32_t slot() const { return core_.slot(); }
  uint64_t slot_bytes() const { return core_.slot_bytes(); }

 private:
  ClientCore core_;
};

}  // namespace
PYBIND11_MODULE(_host, m) {
  m.doc() = "applestar_amd host runtime: shared-memory request/response channels (futex based)";
  py::class_<ShmServer>(m, "ShmServer")
      .def(py::init<const std::string&, uint32_t, uint64_t>(), py::arg("name"), py::arg("n_slots"),
           py::arg("slot_bytes"))
      .def("wait", &ShmServer::wait, py::arg("timeout_ms") = -1)
      .def("pending", &ShmServer::pending)
      .def("request", &ShmServer::request)
      .def("tag", &ShmServer::tag)
      .def("respond", &ShmServer::respond)
      .def("dead_slots", &ShmServer::dead_slots)
      .def("close", &ShmServer::close)
      .def_property_readonly("name", &ShmServer::name)
      .def_property_readonly("n_slots", &ShmServer::n_slots)
      .def_property_readonly("slot_bytes", &ShmServer::slot_bytes)
      .def_property_readonly("base_address", &ShmServer::base_address)
      .def_property_readonly("size", &ShmServer::size);
  py::class_<ShmClient>(m, "ShmClient")
      .def(py::init<const std::string&, uint32_t, uint32_t>(), py::arg("name"), py::arg("slot"),
           py::arg("tag") = 0)
      .def("request", &ShmClient::request, py::arg("data"), py::arg("timeout_ms") = -1)
      .def_property_readonly("slot", &ShmClient::slot)
      .def_property_readonly("slot_bytes", &ShmClient::slot_bytes);
}
