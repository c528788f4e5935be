/* _nhaddr -- data addresses of contiguous host buffers for the ctypes shim.
 *
 * The per-block drop-in path (nano_hevc.intra / transform / quant / metrics)
 * hands 2-4 numpy arrays to the C ABI per call.  numpy's own routes to a data
 * pointer (arr.ctypes.data_as, arr.ctypes.data, __array_interface__) build
 * helper objects and cost 1-4 us each -- more than the GPU round trip of a
 * block-sized call.  addr(*arrays) returns the buffer address of each argument
 * through the buffer protocol (PyObject_GetBuffer, C-contiguous, ~0.1 us): an
 * int (or a tuple of ints) the ctypes call takes as c_void_p.
 *
 * Host glue only: no arithmetic, no device code.  Built in-tree by
 * nano-hevc_amd/Makefile with the system compiler against this interpreter's
 * headers; nano_hevc/_lib.py falls back to numpy's ctypes route without it.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

static int one_addr(PyObject* o, PyObject** out) {
    Py_buffer view;
    if (PyObject_GetBuffer(o, &view, PyBUF_C_CONTIGUOUS) != 0) return -1;
    *out = PyLong_FromVoidPtr(view.buf);
    PyBuffer_Release(&view);
    return *out ? 0 : -1;
}

static PyObject* nh_addr(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    (void)self;
    if (nargs == 1) {
        PyObject* r = NULL;
        return one_addr(args[0], &r) ? NULL : r;
    }
    PyObject* t = PyTuple_New(nargs);
    if (!t) return NULL;
    for (Py_ssize_t i = 0; i < nargs; ++i) {
        PyObject* r = NULL;
        if (one_addr(args[i], &r)) {
            Py_DECREF(t);
            return NULL;
        }
        PyTuple_SET_ITEM(t, i, r);
    }
    return t;
}

static PyMethodDef methods[] = {
    {"addr", (PyCFunction)(void (*)(void))nh_addr, METH_FASTCALL,
     "addr(a[, b, ...]) -> data address(es) of C-contiguous buffers"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_nhaddr", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__nhaddr(void) { return PyModule_Create(&module); }
