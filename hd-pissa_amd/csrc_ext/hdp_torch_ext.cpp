// Host runtime of the module backward -> grouped probe (K2) path, bound to torch tensors.
//
// The reference's module backward is autograd's (hp:139): per CustomLinearLayer, per micro-step,
// a handful of ATen launches.  Here every module backward only PUSHES (X, G) onto the native
// probe queue (include/hdpissa.h hdp_probe_queue_*) and the queue launches one grouped sweep per
// backward pass.  The push is on the host critical path of every module of every micro-step
// (1,792 per LLaMA-2-7B step at 8 micro-batches), so it is native: tensor checks, the current
// HIP stream, the C-ABI call and the lifetime of the pushed activations (kept alive until the
// group that reads them is launched) cost ~1 us here instead of ~10 us through Python + ctypes.
//
// This file only binds torch tensors to the C-ABI; every kernel lives in libhdpissa.so.
#include <torch/extension.h>
#include <c10/hip/HIPStream.h>

#include <unordered_set>
#include <vector>

#include "hdpissa.h"

namespace {

void check(int rc, const char* what) {
  if (rc != HDP_OK) TORCH_CHECK(false, what, " failed (status ", rc, "): ", hdp_last_error());
}

class ProbeQueue {
 public:
  ProbeQueue(bool bf16, int max_items, int64_t budget_bytes) : dtype_(bf16 ? HDP_BF16 : HDP_F32) {
    check(hdp_probe_queue_create(dtype_, max_items, budget_bytes, &q_), "hdp_probe_queue_create");
  }
  ~ProbeQueue() { close(); }

  int add_module(int64_t A, int64_t Bt, int64_t gA, int64_t gB, int64_t in, int64_t out, int r, double scale) {
    int slot = -1;
    check(hdp_probe_queue_add_module(q_, reinterpret_cast<const float*>(A), reinterpret_cast<const float*>(Bt), 1,
                                     reinterpret_cast<float*>(gA), reinterpret_cast<float*>(gB), in, out, r,
                                     (float)scale, &slot),
          "hdp_probe_queue_add_module");
    return slot;
  }

  // X: [..., in], G: [..., out] in the queue's dtype (G of another float dtype is converted).
  // Returns true if the push launched the previously pending group first.
  bool push(int slot, const at::Tensor& x, const at::Tensor& gy, bool accumulate, int64_t in, int64_t out) {
    TORCH_CHECK(q_ != nullptr, "probe queue closed");
    at::Tensor X = x, G = gy;
    if (!X.is_contiguous()) X = X.contiguous();
    if (G.scalar_type() != X.scalar_type()) G = G.to(X.scalar_type());
    if (!G.is_contiguous()) G = G.contiguous();
    const int want = X.scalar_type() == at::kBFloat16 ? HDP_BF16 : HDP_F32;
    TORCH_CHECK(want == dtype_ && (X.scalar_type() == at::kFloat || X.scalar_type() == at::kBFloat16),
                "probe queue dtype mismatch");
    TORCH_CHECK(X.is_cuda() && G.is_cuda(), "hdpissa_amd HIP ops need tensors on a HIP device (no CPU fallback)");
    TORCH_CHECK(X.numel() % in == 0 && G.numel() % out == 0 && X.numel() / in == G.numel() / out,
                "probe push: shape mismatch");
    // the kernels load 16-byte granules: re-base a view at an odd storage offset
    if (reinterpret_cast<uintptr_t>(X.data_ptr()) & 15) X = X.clone();
    if (reinterpret_cast<uintptr_t>(G.data_ptr()) & 15) G = G.clone();
    const int64_t T = in > 0 ? X.numel() / in : 0;
    void* stream = c10::hip::getCurrentHIPStream(X.device().index()).stream();
    int flushed = 0;
    check(hdp_probe_queue_push(q_, slot, X.data_ptr(), G.data_ptr(), T, accumulate ? 1 : 0, stream, &flushed),
          "hdp_probe_queue_push");
    if (flushed) {
      held_.clear();
      slots_.clear();
    }
    held_.push_back(X);
    held_.push_back(G);
    slots_.insert(slot);
    return flushed != 0;
  }

  void flush() {
    if (q_ == nullptr || held_.empty()) return;
    check(hdp_probe_queue_flush(q_), "hdp_probe_queue_flush");
    held_.clear();
    slots_.clear();
  }

  bool pending_slot(int slot) const { return slots_.count(slot) != 0; }
  int pending() const { return q_ ? hdp_probe_queue_pending(q_) : 0; }
  int64_t flushes() const { return q_ ? hdp_probe_queue_flushes(q_) : 0; }
  int64_t handle() const { return reinterpret_cast<int64_t>(q_); }

  void close() {
    if (q_ == nullptr) return;
    try {
      flush();
    } catch (...) {
    }
    hdp_probe_queue_destroy(q_);
    q_ = nullptr;
    held_.clear();
    slots_.clear();
  }

 private:
  int dtype_;
  hdp_probe_queue q_ = nullptr;
  std::vector<at::Tensor> held_;   // pushed X / G: alive until their group is launched
  std::unordered_set<int> slots_;  // modules in the pending group
};

}  // namespace

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "torch binding of libhdpissa's native probe queue (module backward -> grouped K2)";
  pybind11::class_<ProbeQueue>(m, "ProbeQueue")
      .def(pybind11::init<bool, int, int64_t>())
      .def("add_module", &ProbeQueue::add_module)
      .def("push", &ProbeQueue::push)
      .def("flush", &ProbeQueue::flush)
      .def("pending_slot", &ProbeQueue::pending_slot)
      .def("pending", &ProbeQueue::pending)
      .def("flushes", &ProbeQueue::flushes)
      .def("handle", &ProbeQueue::handle)
      .def("close", &ProbeQueue::close);
}
