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
#include <c10/hip/HIPCachingAllocator.h>
#include <c10/hip/HIPStream.h>
#include <torch/csrc/autograd/engine.h>
#include <torch/csrc/autograd/graph_task.h>
#include <torch/csrc/autograd/python_variable.h>

#include <optional>
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
    const c10::hip::HIPStream cur = c10::hip::getCurrentHIPStream(X.device().index());
    void* stream = cur.stream();
    int flushed = 0;
    check(hdp_probe_queue_push(q_, slot, X.data_ptr(), G.data_ptr(), T, accumulate ? 1 : 0, stream, &flushed),
          "hdp_probe_queue_push");
    if (flushed) release(cur);  // the previous group was launched (on its own stream)
    stream_ = cur;
    held_.push_back(X);
    held_.push_back(G);
    slots_.insert(slot);
    return flushed != 0;
  }

  void flush() {
    if (q_ == nullptr || held_.empty()) return;
    check(hdp_probe_queue_flush(q_), "hdp_probe_queue_flush");
    release(c10::hip::getCurrentHIPStream(stream_ ? stream_->device_index() : -1));
  }

  // end of the running backward pass (autograd engine callback, once per graph task): launch the
  // pending group so A.grad / B.grad are complete when backward() returns
  void flush_at_end_of_backward() {
    const int task = torch::autograd::get_current_graph_task_id();
    if (task == -1 || task == cb_task_) return;
    cb_task_ = task;
    torch::autograd::Engine::get_default_engine().queue_callback([this] { flush(); });
  }

  int dtype() const { return dtype_; }
  bool closed() const { return q_ == nullptr; }
  // LayerSlot pushes allowed (off once the arena has a second dtype's queue: the Python path then
  // launches the other queue's pending group before each push, keeping push order)
  bool fast() const { return fast_ && q_ != nullptr; }
  void set_fast(bool on) { fast_ = on; }

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
  // the pending group has been launched on stream_: drop the pushed X / G.  The caching allocator is
  // told that every block is in use on stream_ (whatever stream allocated it, and whichever stream
  // the caller is on now), so it does not hand a block out before the group's kernels have run (the
  // Python path's record_stream); for a block allocated on stream_ itself the call is a no-op
  void release(const c10::hip::HIPStream& /*now*/) {
    if (stream_)
      for (const at::Tensor& t : held_) c10::hip::HIPCachingAllocator::recordStream(t.storage().data_ptr(), *stream_);
    held_.clear();
    slots_.clear();
  }

  int dtype_;
  std::optional<c10::hip::HIPStream> stream_;  // the stream of the pending pushes
  hdp_probe_queue q_ = nullptr;
  std::vector<at::Tensor> held_;   // pushed X / G: alive until their group is launched
  std::unordered_set<int> slots_;  // modules in the pending group
  int cb_task_ = -1;
  bool fast_ = true;
};

// One adapter layer's fast module-backward push (CustomLinearLayer._probe_backward): everything
// the Python path checks per call -- the layer's A / B are the Parameters it was registered with,
// B unchanged since B^T was cached, A.grad / B.grad both unset (first micro-step: they become the
// arena views, overwrite) or both the arena views (accumulate), the activation dtype is this
// queue's -- then the native push and the end-of-backward flush.  Returns false (nothing done)
// whenever the Python path must decide, so edge cases keep the reference's behaviour.
class LayerSlot {
 public:
  LayerSlot(pybind11::object queue, int slot, pybind11::object A, pybind11::object B, at::Tensor gA, at::Tensor gB,
            int64_t in, int64_t out, int64_t b_version)
      : queue_obj_(std::move(queue)), slot_(slot), A_(std::move(A)), B_(std::move(B)), gA_(std::move(gA)),
        gB_(std::move(gB)), in_(in), out_(out), b_version_(b_version) {
    q_ = queue_obj_.cast<ProbeQueue*>();
    want_ = q_->dtype() == HDP_BF16 ? at::kBFloat16 : at::kFloat;
  }

  bool push(pybind11::handle params, const at::Tensor& x, const at::Tensor& gy) {
    PyObject* d = params.ptr();
    if (!q_->fast() || !PyDict_Check(d)) return false;
    PyObject* A = PyDict_GetItemString(d, "A");
    PyObject* B = PyDict_GetItemString(d, "B");
    if (A != A_.ptr() || B != B_.ptr() || !THPVariable_Check(A) || !THPVariable_Check(B)) return false;
    const at::Tensor& At = THPVariable_Unpack(A);
    const at::Tensor& Bt = THPVariable_Unpack(B);
    if (Bt._version() != b_version_) return false;
    if (x.scalar_type() != want_ || !x.is_cuda()) return false;
    const at::Tensor& ga = At.grad();
    const at::Tensor& gb = Bt.grad();
    bool accumulate;
    if (!ga.defined() && !gb.defined()) {
      accumulate = false;
    } else if (ga.defined() && gb.defined() && ga.data_ptr() == gA_.data_ptr() && gb.data_ptr() == gB_.data_ptr()) {
      accumulate = true;
    } else {
      return false;
    }
    q_->push(slot_, x, gy, accumulate, in_, out_);  // may throw: the grads stay as they were
    if (!accumulate) {  // first micro-step: A.grad / B.grad become the arena views the group overwrites
      const_cast<at::Tensor&>(At).mutable_grad() = gA_;
      const_cast<at::Tensor&>(Bt).mutable_grad() = gB_;
    }
    q_->flush_at_end_of_backward();
    return true;
  }

 private:
  pybind11::object queue_obj_;  // keeps the queue alive
  ProbeQueue* q_ = nullptr;
  int slot_;
  pybind11::object A_, B_;
  at::Tensor gA_, gB_;
  int64_t in_, out_, b_version_;
  at::ScalarType want_;
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
      .def("close", &ProbeQueue::close)
      .def("set_fast", &ProbeQueue::set_fast);
  pybind11::class_<LayerSlot>(m, "LayerSlot")
      .def(pybind11::init<pybind11::object, int, pybind11::object, pybind11::object, at::Tensor, at::Tensor, int64_t,
                          int64_t, int64_t>())
      .def("push", &LayerSlot::push);
}
