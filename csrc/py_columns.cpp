// ``cat_dict_columns(items, keys, widths)``: MeanAveragePrecision's batched update (reference
// ``detection/mean_ap.py:458-499`` appends every image's dict entries one by one) reads each column of a list of
// per-image dicts -- boxes / scores / labels, [k, 4] or [k] -- straight from the Python objects.
//
// Why a CPython entry point and not a ``torch.ops`` op: boxing a ``Tensor[]`` argument of 512 tensors into the
// dispatcher's IValue list costs ~200 us on the host (measured: an op with an empty body), the per-tensor checks a
// few us.  Here every dict value is unpacked in place (``THPVariable_Unpack``: a reference, no refcount traffic), one
// pass checks the whole batch -- one dtype / device per column, 1-d (width 0) or [k, width], no autograd, k > 0, the
// same row count k for every column of an item -- and each column becomes a view of its storage when the items are
// consecutive contiguous row blocks of one tensor (a data loader's batch tensor indexed per image), else one at::cat.
//
// Returns ``None`` when the batch is not uniform (the caller's per-image path validates it with the reference's
// messages), else ``([flat per key], [k per item])``.  ``widths[c] < 0`` marks an optional column (width
// ``-widths[c] - 1``): present in every item or in none (``None`` in the result), anything else is ``None`` overall.
// The module init shares the library file with the ``torch.ops.tmx`` registrations (``ops.py_module()``).
#include <Python.h>

#include <ATen/ATen.h>
#include <torch/csrc/autograd/python_variable.h>

#include <vector>

namespace {

struct Column {
  PyObject* key = nullptr;
  int64_t width = 0;
  bool optional = false;
  int present = -1;  // -1 undecided, 0 absent in every item, 1 present in every item
  at::ScalarType dtype = at::ScalarType::Undefined;
  at::Device device = at::Device(at::kCPU);
  const void* storage = nullptr;
  const char* next = nullptr;
  bool chained = true;
  int64_t total = 0;
  std::vector<const at::Tensor*> items;
};

PyObject* not_uniform() { Py_RETURN_NONE; }

PyObject* cat_dict_columns(PyObject*, PyObject* args) {
  PyObject *items, *keys, *widths;
  if (!PyArg_ParseTuple(args, "OOO", &items, &keys, &widths)) return nullptr;
  if (!PyList_CheckExact(items) || !PyTuple_CheckExact(keys) || !PyTuple_CheckExact(widths) ||
      PyTuple_GET_SIZE(keys) != PyTuple_GET_SIZE(widths)) {
    PyErr_SetString(PyExc_TypeError, "cat_dict_columns(list, tuple of str, tuple of int)");
    return nullptr;
  }
  const Py_ssize_t n = PyList_GET_SIZE(items), nk = PyTuple_GET_SIZE(keys);
  if (n == 0 || nk == 0) return not_uniform();
  std::vector<Column> cols(static_cast<size_t>(nk));
  for (Py_ssize_t c = 0; c < nk; ++c) {
    const long w = PyLong_AsLong(PyTuple_GET_ITEM(widths, c));
    if (w == -1 && PyErr_Occurred()) return nullptr;
    cols[c].key = PyTuple_GET_ITEM(keys, c);
    cols[c].optional = w < 0;
    cols[c].width = w < 0 ? -w - 1 : w;
    cols[c].items.reserve(static_cast<size_t>(n));
  }
  std::vector<int64_t> rows(static_cast<size_t>(n));
  try {
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* d = PyList_GET_ITEM(items, i);
      if (!PyDict_Check(d)) return not_uniform();
      int64_t k_item = -1;
      for (Py_ssize_t c = 0; c < nk; ++c) {
        Column& col = cols[c];
        PyObject* v = PyDict_GetItemWithError(d, col.key);  // borrowed
        if (v == nullptr) {
          if (PyErr_Occurred()) return nullptr;
          if (!col.optional || col.present == 1) return not_uniform();
          col.present = 0;
          continue;
        }
        if (col.present == 0) return not_uniform();
        if (!THPVariable_Check(v)) return not_uniform();
        const at::Tensor& t = THPVariable_Unpack(v);
        const at::TensorImpl* ti = t.unsafeGetTensorImpl();
        const int64_t want_dim = col.width > 0 ? 2 : 1;
        if (ti->dim() != want_dim || (col.width > 0 && ti->size(1) != col.width) || t.requires_grad()) return not_uniform();
        const int64_t k = ti->size(0);
        if (k == 0) return not_uniform();  // (empty images take the per-item path, as the reference's loop)
        if (k_item < 0) k_item = k;
        else if (k != k_item) return not_uniform();
        if (col.present < 0) {
          col.present = 1;
          col.dtype = t.scalar_type();
          col.device = t.device();
          col.storage = ti->storage().data();
        } else if (t.scalar_type() != col.dtype || t.device() != col.device) {
          return not_uniform();
        }
        if (col.chained) {
          const char* p = static_cast<const char*>(ti->data());
          col.chained = ti->is_contiguous() && ti->storage().data() == col.storage && (col.next == nullptr || p == col.next);
          col.next = p + k * (col.width > 0 ? col.width : 1) * static_cast<int64_t>(t.element_size());
        }
        col.total += k;
        col.items.push_back(&t);
      }
      if (k_item < 0) return not_uniform();  // an item with no column at all
      rows[i] = k_item;
    }
    PyObject* flats = PyList_New(nk);
    if (flats == nullptr) return nullptr;
    for (Py_ssize_t c = 0; c < nk; ++c) {
      Column& col = cols[c];
      PyObject* obj;
      if (col.present != 1) {
        Py_INCREF(Py_None);
        obj = Py_None;
      } else {
        at::Tensor flat;
        const at::Tensor& first = *col.items.front();
        if (col.chained) {
          std::vector<int64_t> shape = {col.total};
          std::vector<int64_t> stride = {col.width > 0 ? col.width : 1};
          if (col.width > 0) {
            shape.push_back(col.width);
            stride.push_back(1);
          }
          flat = first.as_strided(shape, stride, first.storage_offset());
        } else {
          std::vector<at::Tensor> parts;
          parts.reserve(col.items.size());
          for (const at::Tensor* t : col.items) parts.push_back(*t);
          flat = at::cat(parts, 0);
        }
        obj = THPVariable_Wrap(std::move(flat));
        if (obj == nullptr) {
          Py_DECREF(flats);
          return nullptr;
        }
      }
      PyList_SET_ITEM(flats, c, obj);
    }
    PyObject* sizes = PyList_New(n);
    if (sizes == nullptr) {
      Py_DECREF(flats);
      return nullptr;
    }
    for (Py_ssize_t i = 0; i < n; ++i) {
      PyObject* k = PyLong_FromLongLong(rows[i]);
      if (k == nullptr) {
        Py_DECREF(flats);
        Py_DECREF(sizes);
        return nullptr;
      }
      PyList_SET_ITEM(sizes, i, k);
    }
    return Py_BuildValue("(NN)", flats, sizes);
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
}

PyMethodDef kMethods[] = {
    {"cat_dict_columns", cat_dict_columns, METH_VARARGS,
     "cat_dict_columns(items, keys, widths) -> None | ([flat per key], [rows per item])"},
    {nullptr, nullptr, 0, nullptr},
};

PyModuleDef kModule = {PyModuleDef_HEAD_INIT, "_tmx_native", "host-side helpers of the torchmetrics_forked_amd native library",
                       -1, kMethods, nullptr, nullptr, nullptr, nullptr};

}  // namespace

PyMODINIT_FUNC PyInit__tmx_native() { return PyModule_Create(&kModule); }
