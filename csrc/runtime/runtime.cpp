// Native runtime pieces of faster_distributed_training_amd (C++ / HIP runtime API).
//
// * PinnedPrefetcher — the MI355X replacement for the reference's DataLoader
//   pin-memory thread + prefetch_generator.BackgroundGenerator + `.to(device,
//   non_blocking=True)` (resnet50_test.py:41-43,522; transformer_test.py:68-70,242-245):
//   a ring of pinned host slots (hipHostMalloc), a dedicated non-blocking HIP copy
//   stream, and one hipEvent per slot.  `stage()` memcpy's a host batch into a free
//   slot (GIL released) and enqueues hipMemcpyAsync H2D on the copy stream;
//   `wait()` makes the compute stream wait on that event (hipStreamWaitEvent), so the
//   H2D transfer overlaps compute of the previous step and the host never blocks on
//   the GPU except when the ring is full.
// * plan_buckets — gradient bucket assignment for the DDP reducer (parallel/ddp.py):
//   parameters in reverse registration order (≈ backward order), a small first bucket
//   so communication starts early in backward, then `cap` bytes per bucket.  Sized for
//   RCCL over xGMI (7 point-to-point links/GPU): see parallel/ddp.py.
#include <hip/hip_runtime.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <vector>

#include "ordered_worker.h"
#include "runtime_api.h"

namespace py = pybind11;

namespace fdt {

#define RT_CHECK(expr)                                                                     \
  do {                                                                                     \
    hipError_t _e = (expr);                                                                \
    if (_e != hipSuccess) throw std::runtime_error(std::string(#expr) + ": " + hipGetErrorString(_e)); \
  } while (0)

class PinnedPrefetcher {
 public:
  PinnedPrefetcher(int device, size_t slot_bytes, int nslots) : device_(device), slot_bytes_(slot_bytes) {
    if (nslots < 2) throw std::runtime_error("PinnedPrefetcher needs >= 2 slots");
    RT_CHECK(hipSetDevice(device_));
    RT_CHECK(hipStreamCreateWithFlags(&copy_stream_, hipStreamNonBlocking));
    slots_.resize(nslots, nullptr);
    events_.resize(nslots, nullptr);
    used_.resize(nslots, 0);
    slot_seq_.resize(nslots, 0);
    for (int i = 0; i < nslots; ++i) {
      RT_CHECK(hipHostMalloc(&slots_[i], slot_bytes_, hipHostMallocDefault));
      RT_CHECK(hipEventCreateWithFlags(&events_[i], hipEventDisableTiming));
    }
  }
  ~PinnedPrefetcher() {
    worker_.reset();  // drains the queued jobs, joins the thread
    hipSetDevice(device_);
    if (copy_stream_) hipStreamSynchronize(copy_stream_);
    for (auto e : events_) if (e) hipEventDestroy(e);
    for (auto p : slots_) if (p) hipHostFree(p);
    if (copy_stream_) hipStreamDestroy(copy_stream_);
  }

  // Copy `nbytes` from host address `src` into the next ring slot, then enqueue the
  // H2D copy into device address `dst`.  Returns the slot id to pass to wait().
  int stage(uint64_t src, size_t nbytes, uint64_t dst) {
    if (nbytes > slot_bytes_) throw std::runtime_error("PinnedPrefetcher: batch larger than slot");
    const int s = next_;
    next_ = (next_ + 1) % (int)slots_.size();
    {
      py::gil_scoped_release nogil;
      RT_CHECK(hipSetDevice(device_));
      if (used_[s]) RT_CHECK(hipEventSynchronize(events_[s]));  // slot's previous copy done
      std::memcpy(slots_[s], reinterpret_cast<const void*>(src), nbytes);
      RT_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dst), slots_[s], nbytes, hipMemcpyHostToDevice, copy_stream_));
      RT_CHECK(hipEventRecord(events_[s], copy_stream_));
      used_[s] = 1;
    }
    return s;
  }

  // Stage several (src, nbytes, dst) segments into one slot (e.g. tokens+labels+mask).
  int stage_many(const std::vector<uint64_t>& srcs, const std::vector<size_t>& sizes, const std::vector<uint64_t>& dsts) {
    size_t total = 0;
    for (auto n : sizes) total += (n + 255) / 256 * 256;
    if (total > slot_bytes_) throw std::runtime_error("PinnedPrefetcher: batch larger than slot");
    const int s = next_;
    next_ = (next_ + 1) % (int)slots_.size();
    {
      py::gil_scoped_release nogil;
      RT_CHECK(hipSetDevice(device_));
      if (used_[s]) RT_CHECK(hipEventSynchronize(events_[s]));
      size_t off = 0;
      char* base = static_cast<char*>(slots_[s]);
      for (size_t i = 0; i < srcs.size(); ++i) {
        std::memcpy(base + off, reinterpret_cast<const void*>(srcs[i]), sizes[i]);
        RT_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(dsts[i]), base + off, sizes[i], hipMemcpyHostToDevice,
                                copy_stream_));
        off += (sizes[i] + 255) / 256 * 256;
      }
      RT_CHECK(hipEventRecord(events_[s], copy_stream_));
      used_[s] = 1;
    }
    return s;
  }

  // Background form of stage_many: queue the job (slot-reuse wait, memcpy into the pinned
  // slot, H2D enqueue) to the worker thread and return the slot at once.  `wait_event`
  // (a hipEvent_t, or 0) is waited on by the copy stream before the H2D: the compute
  // stream's release of the slot's device buffer.  The caller keeps the source arrays and
  // the event alive until wait(s) returned.
  int submit(const std::vector<uint64_t>& srcs, const std::vector<size_t>& sizes, const std::vector<uint64_t>& dsts,
             uint64_t wait_event) {
    if (srcs.size() != sizes.size() || srcs.size() != dsts.size())
      throw std::runtime_error("PinnedPrefetcher.submit: srcs / sizes / dsts lengths differ");
    size_t total = 0;
    for (auto n : sizes) total += (n + 255) / 256 * 256;
    if (total > slot_bytes_) throw std::runtime_error("PinnedPrefetcher: batch larger than slot");
    const int s = next_;
    next_ = (next_ + 1) % (int)slots_.size();
    if (!worker_) worker_ = std::make_unique<OrderedWorker<Job>>([this](Job& j) { issue(j); });
    slot_seq_[s] = worker_->submit(Job{s, srcs, sizes, dsts, wait_event});
    return s;
  }

  // Make `compute_stream` wait for slot `s`'s H2D copy (no host blocking on the copy; with
  // submit() the call first waits, GIL released, until the worker has issued slot s's job).
  void wait(int s, uint64_t compute_stream) {
    if (s < 0 || s >= (int)slots_.size()) throw std::runtime_error("PinnedPrefetcher.wait: bad slot");
    if (worker_) {
      py::gil_scoped_release nogil;
      worker_->wait_issued(slot_seq_[s]);
    }
    RT_CHECK(hipStreamWaitEvent(reinterpret_cast<hipStream_t>(compute_stream), events_.at(s), 0));
  }
  // Host-only: block (GIL released) until the worker has issued slot `s`'s last job, i.e. its
  // memcpy from the caller's source arrays is done and they may be dropped.
  void wait_issued(int s) {
    if (s < 0 || s >= (int)slots_.size()) throw std::runtime_error("PinnedPrefetcher.wait_issued: bad slot");
    if (worker_) {
      py::gil_scoped_release nogil;
      worker_->wait_issued(slot_seq_[s]);
    }
  }
  uint64_t submitted() const { return worker_ ? worker_->submitted() : 0; }
  void synchronize() {
    if (worker_) {
      py::gil_scoped_release nogil;
      worker_->drain();
    }
    RT_CHECK(hipStreamSynchronize(copy_stream_));
  }
  uint64_t copy_stream() const { return reinterpret_cast<uint64_t>(copy_stream_); }
  size_t slot_bytes() const { return slot_bytes_; }
  int num_slots() const { return (int)slots_.size(); }

 private:
  struct Job {
    int slot;
    std::vector<uint64_t> srcs;
    std::vector<size_t> sizes;
    std::vector<uint64_t> dsts;
    uint64_t wait_event;
  };

  // runs on the worker thread, jobs in submission order (the copy stream sees that order)
  void issue(Job& j) {
    RT_CHECK(hipSetDevice(device_));
    if (j.wait_event) RT_CHECK(hipStreamWaitEvent(copy_stream_, reinterpret_cast<hipEvent_t>(j.wait_event), 0));
    if (used_[j.slot]) RT_CHECK(hipEventSynchronize(events_[j.slot]));  // pinned slot's last H2D done
    size_t off = 0;
    char* base = static_cast<char*>(slots_[j.slot]);
    for (size_t i = 0; i < j.srcs.size(); ++i) {
      std::memcpy(base + off, reinterpret_cast<const void*>(j.srcs[i]), j.sizes[i]);
      RT_CHECK(hipMemcpyAsync(reinterpret_cast<void*>(j.dsts[i]), base + off, j.sizes[i], hipMemcpyHostToDevice,
                              copy_stream_));
      off += (j.sizes[i] + 255) / 256 * 256;
    }
    RT_CHECK(hipEventRecord(events_[j.slot], copy_stream_));
    used_[j.slot] = 1;
  }

  int device_;
  size_t slot_bytes_;
  hipStream_t copy_stream_ = nullptr;
  std::vector<void*> slots_;
  std::vector<hipEvent_t> events_;
  std::vector<char> used_;           // (not vector<bool>: the worker thread writes it)
  int next_ = 0;
  std::vector<uint64_t> slot_seq_;   // worker sequence number of the job last submitted per slot
  std::unique_ptr<OrderedWorker<Job>> worker_;  // background mode (submit); one mode per prefetcher
};

// Device properties needed by the Python side without initialising torch.cuda.
py::dict device_info(int device) {
  hipDeviceProp_t p;
  RT_CHECK(hipGetDeviceProperties(&p, device));
  py::dict d;
  d["name"] = std::string(p.gcnArchName);
  d["cus"] = p.multiProcessorCount;
  d["lds_per_cu"] = (long)p.maxSharedMemoryPerMultiProcessor;
  d["l2"] = p.l2CacheSize;
  d["hbm_bytes"] = (long long)p.totalGlobalMem;
  d["clock_khz"] = p.clockRate;
  return d;
}

void register_runtime(py::module_& m) {
  py::class_<PinnedPrefetcher>(m, "PinnedPrefetcher")
      .def(py::init<int, size_t, int>(), py::arg("device"), py::arg("slot_bytes"), py::arg("nslots") = 3)
      .def("stage", &PinnedPrefetcher::stage)
      .def("stage_many", &PinnedPrefetcher::stage_many)
      .def("submit", &PinnedPrefetcher::submit, py::arg("srcs"), py::arg("sizes"), py::arg("dsts"),
           py::arg("wait_event") = 0)
      .def_property_readonly("submitted", &PinnedPrefetcher::submitted)
      .def("wait", &PinnedPrefetcher::wait)
      .def("wait_issued", &PinnedPrefetcher::wait_issued)
      .def("synchronize", &PinnedPrefetcher::synchronize)
      .def_property_readonly("copy_stream", &PinnedPrefetcher::copy_stream)
      .def_property_readonly("slot_bytes", &PinnedPrefetcher::slot_bytes)
      .def_property_readonly("num_slots", &PinnedPrefetcher::num_slots);
  m.def("plan_buckets", &plan_buckets, py::arg("sizes"), py::arg("first_cap"), py::arg("cap"));
  m.def("device_info", &device_info, py::arg("device") = 0);
}

}  // namespace fdt
