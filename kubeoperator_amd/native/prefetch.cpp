// Native token prefetcher for the training chart's data path (TokenFileDataset).
//
// The flat token file (uint16 or uint32 ids, the usual pre-tokenised corpus layout) is memory-mapped once;
// a pool of worker threads fills a ring of batches ahead of the training loop, each batch = `batch` random
// windows of `window` tokens widened to int64 (the embedding's index dtype), so the Python step only pins
// and copies. Batch i is a pure function of (seed, i): the random starts come from splitmix64(seed, i, row),
// so the stream is reproducible and independent of thread timing, and resuming at step k only needs
// `skip(k * accum)`. madvise(MADV_RANDOM) keeps the kernel from reading ahead megabytes per window.
//
// There is no reference counterpart (the reference ships no training workload): this is the
// MI355X build's native data-loader component.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "prefetch_core.h"

namespace py = pybind11;
using kop_native::TokenPrefetcher;

PYBIND11_MODULE(prefetch, m) {
  m.doc() = "Native multi-threaded token-window prefetcher over a memory-mapped token file";
  py::class_<TokenPrefetcher>(m, "TokenPrefetcher")
      .def(py::init<const std::string&, int, int64_t, int64_t, uint64_t, int, int>(), py::arg("path"),
           py::arg("itemsize"), py::arg("batch"), py::arg("window"), py::arg("seed") = 0, py::arg("depth") = 8,
           py::arg("threads") = 4)
      .def("next",
           [](TokenPrefetcher& self) {
             std::vector<int64_t> v;
             {
               py::gil_scoped_release nogil;
               v = self.next();
             }
             auto* heap = new std::vector<int64_t>(std::move(v));
             py::capsule owner(heap, [](void* p) { delete static_cast<std::vector<int64_t>*>(p); });
             return py::array_t<int64_t>({self.batch(), self.window()}, {self.window() * 8, (int64_t)8}, heap->data(),
                                         owner);
           })
      .def("skip", &TokenPrefetcher::skip)
      .def("starts", &TokenPrefetcher::starts)
      .def_property_readonly("num_tokens", &TokenPrefetcher::num_tokens)
      .def_property_readonly("position", &TokenPrefetcher::position);
}
