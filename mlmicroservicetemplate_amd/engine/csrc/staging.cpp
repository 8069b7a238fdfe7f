// Host staging for the per-GPU engine (T4): gather a batch of per-request sample buffers into
// one pinned slot with a persistent pool of copy threads.
//
// The engine's submit() path used a Python ThreadPoolExecutor (4 threads, one future per quarter
// of the batch): ~0.33-0.5 ms for a ResNet-50 batch (32 x 150 KB = 4.8 MB) -- 10-15 GB/s, and
// the main thread paid the executor round trip on every batch.  Here the copy runs with the GIL
// released on threads that live as long as the engine: the caller hands over (dst, srcs) and
// takes a share of the chunks itself, so there is no wake-up latency on the critical path when
// the workers are slow to start.  Chunks are <= 256 KiB slices of the requests, taken from an
// atomic cursor (a slow or descheduled thread cannot hold up the whole batch).
//
// Threads inherit the CPU affinity of the thread that creates the pool (the engine is built
// after parallel/affinity.bind_to_gpu, so the copies run on the GPU's NUMA node).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

#include "staging_core.h"

namespace py = pybind11;

namespace {

using mls_staging::Stager;

// srcs: a list of C-contiguous numpy arrays of exactly `each` bytes (checked under the GIL).
void gather_arrays(Stager& st, uintptr_t dst, const py::list& srcs, size_t each) {
  std::vector<uintptr_t> ptrs;
  ptrs.reserve(srcs.size());
  for (const auto& o : srcs) {
    py::array a = py::reinterpret_borrow<py::array>(o);
    if (!(a.flags() & py::array::c_style)) throw std::invalid_argument("sample is not C-contiguous");
    if (static_cast<size_t>(a.nbytes()) != each)
      throw std::invalid_argument("sample has " + std::to_string(a.nbytes()) + " bytes, expected " +
                                  std::to_string(each));
    ptrs.push_back(reinterpret_cast<uintptr_t>(a.data()));
  }
  py::gil_scoped_release nogil;
  st.gather(dst, ptrs, each);
}

}  // namespace

PYBIND11_MODULE(_staging, m) {
  m.doc() = "Engine host staging: parallel gather of request buffers into a pinned slot";
  py::class_<Stager>(m, "Stager")
      .def(py::init<int>(), py::arg("threads"))
      .def_property_readonly("threads", &Stager::threads)
      .def("gather", &gather_arrays, py::arg("dst"), py::arg("srcs"), py::arg("each"),
           "Copy each array of `srcs` (C-contiguous, `each` bytes) to dst + i*each; GIL released.")
      .def(
          "gather_ptrs",
          [](Stager& st, uintptr_t dst, const std::vector<uintptr_t>& srcs, size_t each) {
            py::gil_scoped_release nogil;
            st.gather(dst, srcs, each);
          },
          py::arg("dst"), py::arg("srcs"), py::arg("each"));
}
