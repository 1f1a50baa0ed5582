// Host-side dataset index builders (module `smdt_amd._runtime`).
//
// Native replacement for Megatron's `megatron/data/helpers.cpp` as used by the reference's
// GPT dataset (call site /root/reference/3_training_megatron-lm/megatron/data/
// gpt_dataset.py:431-437, Python twin :533-579): packs documents into (seq_length + 1)-token
// samples, and the greedy blending schedule used by BlendableDataset.
//
// Both builders release the GIL; sample_idx switches to int64 automatically when token counts
// exceed int32 (long-running 288 GB-class corpora).
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>

#include <algorithm>
#include <cstdint>
#include <limits>
#include <stdexcept>
#include <vector>

namespace py = pybind11;

namespace {

template <typename IDX>
py::array build_sample_idx_t(const int32_t* sizes, int64_t nsizes, const int32_t* doc_idx, int64_t ndoc,
                             int64_t seq_length, int64_t num_epochs, int64_t tokens_per_epoch) {
  const int64_t num_samples = (num_epochs * tokens_per_epoch - 1) / seq_length;
  std::vector<IDX> out((size_t)(num_samples + 1) * 2);
  {
    py::gil_scoped_release nogil;
    int64_t sample_index = 0, doc_idx_index = 0, doc_offset = 0;
    out[0] = 0;
    out[1] = 0;
    ++sample_index;
    while (sample_index <= num_samples) {
      int64_t remaining = seq_length + 1;
      while (remaining != 0) {
        if (doc_idx_index >= ndoc) throw std::runtime_error("build_sample_idx: ran past doc_idx");
        const int32_t doc_id = doc_idx[doc_idx_index];
        if (doc_id < 0 || doc_id >= nsizes) throw std::runtime_error("build_sample_idx: doc id out of range");
        const int64_t doc_length = (int64_t)sizes[doc_id] - doc_offset;
        remaining -= doc_length;
        if (remaining <= 0) {
          doc_offset += (remaining + doc_length - 1);
          remaining = 0;
        } else {
          ++doc_idx_index;
          doc_offset = 0;
        }
      }
      out[2 * sample_index] = (IDX)doc_idx_index;
      out[2 * sample_index + 1] = (IDX)doc_offset;
      ++sample_index;
    }
  }
  py::array_t<IDX> arr({(py::ssize_t)(num_samples + 1), (py::ssize_t)2});
  std::copy(out.begin(), out.end(), arr.mutable_data());
  return std::move(arr);
}

py::array build_sample_idx(py::array_t<int32_t, py::array::c_style | py::array::forcecast> sizes,
                           py::array_t<int32_t, py::array::c_style | py::array::forcecast> doc_idx,
                           int64_t seq_length, int64_t num_epochs, int64_t tokens_per_epoch) {
  if (seq_length <= 0) throw std::invalid_argument("seq_length must be positive");
  const int64_t num_samples = (num_epochs * tokens_per_epoch - 1) / seq_length;
  const bool wide = num_epochs * tokens_per_epoch > (int64_t)std::numeric_limits<int32_t>::max() ||
                    doc_idx.size() > (py::ssize_t)std::numeric_limits<int32_t>::max() ||
                    num_samples > (int64_t)std::numeric_limits<int32_t>::max();
  if (wide)
    return build_sample_idx_t<int64_t>(sizes.data(), sizes.size(), doc_idx.data(), doc_idx.size(), seq_length,
                                       num_epochs, tokens_per_epoch);
  return build_sample_idx_t<int32_t>(sizes.data(), sizes.size(), doc_idx.data(), doc_idx.size(), seq_length,
                                     num_epochs, tokens_per_epoch);
}

// Greedy blending: sample i goes to the dataset whose achieved count lags its target
// weight * (i + 1) the most (ties -> lowest index). Returns (dataset_index uint8,
// dataset_sample_index int64).
py::tuple build_blending_indices(py::array_t<double, py::array::c_style | py::array::forcecast> weights,
                                 int64_t size) {
  const int64_t nd = weights.size();
  if (nd <= 0 || nd > 255) throw std::invalid_argument("1..255 datasets supported");
  py::array_t<uint8_t> didx(size);
  py::array_t<int64_t> dsidx(size);
  const double* w = weights.data();
  uint8_t* d = didx.mutable_data();
  int64_t* s = dsidx.mutable_data();
  {
    py::gil_scoped_release nogil;
    std::vector<int64_t> current(nd, 0);
    for (int64_t i = 0; i < size; ++i) {
      const double denom = std::max((double)(i + 1), 1.0);
      int64_t best = 0;
      double best_err = w[0] * denom - (double)current[0];
      for (int64_t k = 1; k < nd; ++k) {
        const double err = w[k] * denom - (double)current[k];
        if (err > best_err) {
          best_err = err;
          best = k;
        }
      }
      d[i] = (uint8_t)best;
      s[i] = current[best];
      ++current[best];
    }
  }
  return py::make_tuple(didx, dsidx);
}

}  // namespace

void register_supervisor(py::module_& m);
void register_cpu_adam(py::module_& m);

PYBIND11_MODULE(_runtime, m) {
  m.doc() = "smdt_amd host runtime: dataset index builders and the rank supervisor";
  m.def("build_sample_idx", &build_sample_idx, py::arg("sizes"), py::arg("doc_idx"), py::arg("seq_length"),
        py::arg("num_epochs"), py::arg("tokens_per_epoch"));
  m.def("build_blending_indices", &build_blending_indices, py::arg("weights"), py::arg("size"));
  register_supervisor(m);
  register_cpu_adam(m);
}
