// psgd_host — native host helper of the Python mirror (powersgd_amd/powersgd.py).
//
// PowerSGD.aggregate (reference powersgd/powersgd.py:64-74) splits the gradient list by the
// compression mask (:76-84) and hands every tensor's storage to the codec. Doing that in
// Python costs ~0.2 us per tensor for data_ptr() alone and as much again for the dtype /
// device / contiguity checks the reference gets from torch ops (:189, :289) — ~70 us per
// ResNet-50 step, comparable to the whole device step. This helper does the split, the
// checks and the pointer tables in one C++ pass over the list (no torch types cross the
// codec's C ABI: the tables are plain void* arrays handed to libpsgd by address).
#include <torch/extension.h>

#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

// psgd.h dtype codes
c10::ScalarType scalar_type(int code) {
    if (code == 0) return c10::ScalarType::Float;
    if (code == 1) return c10::ScalarType::BFloat16;
    if (code == 2) return c10::ScalarType::Double;
    throw std::invalid_argument("unknown psgd dtype code " + std::to_string(code));
}

struct PtrTable {
    std::vector<std::vector<int64_t>> shapes;
    std::vector<uint8_t> mask;
    c10::ScalarType dtype;
    int device;
    std::vector<void*> comp, unc;

    PtrTable(std::vector<std::vector<int64_t>> shapes_, std::vector<bool> mask_, int dtype_code,
             int device_)
        : shapes(std::move(shapes_)), dtype(scalar_type(dtype_code)), device(device_) {
        if (mask_.size() != shapes.size()) throw std::invalid_argument("mask/shape count mismatch");
        size_t nc = 0;
        for (bool b : mask_) {
            mask.push_back(b ? 1 : 0);
            nc += b ? 1 : 0;
        }
        comp.assign(nc ? nc : 1, nullptr);
        unc.assign(shapes.size() - nc ? shapes.size() - nc : 1, nullptr);
    }

    // Fills both tables from `grads`; returns bit 0 = compressed table changed, bit 1 =
    // uncompressed table changed. Raises like the reference on a bad list.
    int fill(const py::list& grads) {
        const size_t L = shapes.size();
        if (size_t(py::len(grads)) != L)
            throw py::value_error("expected " + std::to_string(L) + " gradients, got " +
                                  std::to_string(py::len(grads)));
        int changed = 0;
        size_t ic = 0, iu = 0;
        for (size_t i = 0; i < L; ++i) {
            PyObject* o = PyList_GET_ITEM(grads.ptr(), i);
            if (!THPVariable_Check(o)) throw py::type_error("gradients must be tensors");
            const at::Tensor& t = THPVariable_Unpack(o);
            if (t.scalar_type() != dtype)
                throw std::runtime_error(std::string("expected scalar type ") + c10::toString(dtype) +
                                         " but found " + c10::toString(t.scalar_type()));
            const c10::Device d = t.device();
            if (!d.is_cuda() || d.index() != device)
                throw std::runtime_error("gradient on " + d.str() + ", codec on cuda:" + std::to_string(device));
            const auto sz = t.sizes();
            const auto& want = shapes[i];
            bool same = sz.size() == want.size();
            for (size_t k = 0; same && k < want.size(); ++k) same = sz[k] == want[k];
            if (!same) throw std::runtime_error("gradient " + std::to_string(i) + " has shape " +
                                                c10::str(sz) + ", parameter shape differs");
            if (!t.is_contiguous())
                throw std::runtime_error(
                    "view size is not compatible with input tensor's size and stride (at least one "
                    "dimension spans across two contiguous subspaces). Use .reshape(...) instead.");
            void* p = t.data_ptr();
            if (mask[i]) {
                changed |= comp[ic] != p ? 1 : 0;
                comp[ic++] = p;
            } else {
                changed |= unc[iu] != p ? 2 : 0;
                unc[iu++] = p;
            }
        }
        return changed;
    }

    uintptr_t comp_addr() const { return reinterpret_cast<uintptr_t>(comp.data()); }
    uintptr_t unc_addr() const { return reinterpret_cast<uintptr_t>(unc.data()); }
};

// Pointer table of a plain list (AllReduce.aggregate, reference :22-31): same checks, one
// dtype and device for all tensors (the reference's torch.cat would raise otherwise).
int fill_list(const py::list& ts, uintptr_t dst_addr, int dtype_code, int device) {
    const c10::ScalarType dtype = scalar_type(dtype_code);
    void** dst = reinterpret_cast<void**>(dst_addr);
    int changed = 0;
    const size_t L = py::len(ts);
    for (size_t i = 0; i < L; ++i) {
        PyObject* o = PyList_GET_ITEM(ts.ptr(), i);
        if (!THPVariable_Check(o)) throw py::type_error("expected tensors");
        const at::Tensor& t = THPVariable_Unpack(o);
        const c10::Device d = t.device();
        if (t.scalar_type() != dtype || !d.is_cuda() || d.index() != device)
            throw std::runtime_error("AllReduce expects tensors of one dtype on one device");
        if (!t.is_contiguous())
            throw std::runtime_error("view size is not compatible with input tensor's size and stride");
        void* p = t.data_ptr();
        changed |= dst[i] != p;
        dst[i] = p;
    }
    return changed;
}

// Output buffer of one aggregate call: a flat tensor in tensor order plus one view per output
// (the reference returns fresh tensors each call, powersgd.py:153 / utils.py:19).
//
// A fresh allocation is cheap, but building 161 views through the dispatcher is not
// (~2 us each from Python or C++ ops): on ResNet-50 that alone exceeded the device step. So
// the previous call's buffer is handed out again — but ONLY when nothing outside this cache
// holds any of its views: for every view the TensorImpl reference count (held by p.grad,
// autograd's saved tensors, containers on the C++ side), the PyObject reference count (Python
// variables, lists) and the storage reference count (derived views, .data, .detach(),
// untyped_storage()) must be back at the values they had when the views were created.
// Anything else gets a new buffer, exactly as the reference's per-call empty_like.
// Views are built without the dispatcher (TensorImpl + sizes/strides over the flat storage).
struct OutputSlab {
    std::vector<std::vector<int64_t>> shapes;
    std::vector<int64_t> offs;
    int64_t numel = 0;
    c10::ScalarType dtype;
    int device;
    at::Tensor flat;
    std::vector<at::Tensor> views;
    std::vector<PyObject*> pyviews;  // owned references
    std::vector<int64_t> base_impl;
    std::vector<Py_ssize_t> base_py;
    int64_t base_storage = 0;
    int64_t fresh = 0;  // buffers allocated (diagnostics / tests)

    OutputSlab(std::vector<std::vector<int64_t>> shapes_, int dtype_code, int device_)
        : shapes(std::move(shapes_)), dtype(scalar_type(dtype_code)), device(device_) {
        for (const auto& s : shapes) {
            offs.push_back(numel);
            int64_t n = 1;
            for (int64_t d : s) n *= d;
            numel += n;
        }
    }
    ~OutputSlab() { drop(); }

    void drop() {
        if (!pyviews.empty() && Py_IsInitialized()) {
            py::gil_scoped_acquire g;
            for (PyObject* o : pyviews) Py_XDECREF(o);
        }
        pyviews.clear();
        views.clear();
    }

    bool free_now() const {
        if (!flat.defined()) return false;
        if (int64_t(flat.storage().use_count()) != base_storage) return false;
        for (size_t i = 0; i < views.size(); ++i) {
            if (int64_t(views[i].use_count()) != base_impl[i]) return false;
            if (Py_REFCNT(pyviews[i]) != base_py[i]) return false;
        }
        return true;
    }

    void rebuild() {
        drop();
        flat = at::empty({std::max<int64_t>(numel, 1)},
                         at::TensorOptions().dtype(dtype).device(device < 0 ? at::Device(at::kCPU)
                                                                             : at::Device(at::kCUDA, device)));
        ++fresh;
        const c10::Storage& st = flat.storage();
        for (size_t i = 0; i < shapes.size(); ++i) {
            auto impl = c10::make_intrusive<c10::TensorImpl>(c10::TensorImpl::VIEW, c10::Storage(st),
                                                              flat.key_set(), flat.dtype());
            const auto& s = shapes[i];
            std::vector<int64_t> strides(s.size(), 1);
            for (int k = int(s.size()) - 2; k >= 0; --k) strides[k] = strides[k + 1] * s[k + 1];
            impl->set_sizes_and_strides(s, strides, offs[i]);
            views.emplace_back(std::move(impl));
        }
        for (auto& v : views) pyviews.push_back(THPVariable_Wrap(v));
        base_storage = int64_t(flat.storage().use_count());
        base_impl.clear();
        base_py.clear();
        for (size_t i = 0; i < views.size(); ++i) {
            base_impl.push_back(int64_t(views[i].use_count()));
            base_py.push_back(Py_REFCNT(pyviews[i]));
        }
    }

    py::list get() {
        if (!free_now()) rebuild();
        py::list out(views.size());
        for (size_t i = 0; i < views.size(); ++i) {
            Py_INCREF(pyviews[i]);
            PyList_SET_ITEM(out.ptr(), i, pyviews[i]);
        }
        return out;
    }
    at::Tensor get_flat() const { return flat; }
    uintptr_t data_ptr() const { return reinterpret_cast<uintptr_t>(flat.data_ptr()); }
};

}  // namespace

PYBIND11_MODULE(_psgd_host, m) {
    m.doc() = "powersgd_amd native host helper: gradient split + pointer tables";
    py::class_<PtrTable>(m, "PtrTable")
        .def(py::init<std::vector<std::vector<int64_t>>, std::vector<bool>, int, int>())
        .def("fill", &PtrTable::fill)
        .def("comp_addr", &PtrTable::comp_addr)
        .def("unc_addr", &PtrTable::unc_addr);
    m.def("fill_list", &fill_list);
    py::class_<OutputSlab>(m, "OutputSlab")
        .def(py::init<std::vector<std::vector<int64_t>>, int, int>())
        .def("get", &OutputSlab::get)
        .def_property_readonly("flat", &OutputSlab::get_flat)
        .def("data_ptr", &OutputSlab::data_ptr)
        .def_readonly("fresh", &OutputSlab::fresh);
}
