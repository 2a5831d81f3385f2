/* fastpath.c — CPython entry points for the per-tensor calls of a training step.
 *
 * Backward hooks call mark_communication_ready once per gradient tensor
 * (bagua-core-py/src/lib.rs:318-327 -> bagua-core-internal/src/lib.rs:300-319).
 * Through ctypes each such call costs about 1 us of argument conversion before the
 * scheduler sees it; these METH_FASTCALL functions take plain ints and bytes and
 * call the same C ABI (include/bagua_core.h), releasing the GIL like ctypes does,
 * since a mark can wait for space on the scheduler's bounded channel.  No torch
 * types cross this boundary: the Python side reads data_ptr / numel / dtype.
 */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "bagua_core.h"

/* (handle, name, event, ptr, num_elem, dtype, device_id) -> the descriptor and the call's
 * plain arguments; 0 on success, -1 with a Python error set */
static int parse_mark(PyObject* const* args, Py_ssize_t nargs, void** handle, const char** name, uint64_t* event,
                      bagua_tensor_t* t) {
    if (nargs != 7) {
        PyErr_SetString(PyExc_TypeError, "expected (handle, name, event, ptr, num_elem, dtype, device_id)");
        return -1;
    }
    /* each conversion is checked before the next: no C-API call runs with an error set */
    *handle = PyLong_AsVoidPtr(args[0]);
    if (PyErr_Occurred()) return -1;
    *name = PyBytes_AsString(args[1]);
    if (!*name) return -1;
    *event = (uint64_t)PyLong_AsUnsignedLongLongMask(args[2]);
    if (PyErr_Occurred()) return -1;
    t->ptr = (uint64_t)PyLong_AsUnsignedLongLongMask(args[3]);
    if (PyErr_Occurred()) return -1;
    t->num_elem = (uint64_t)PyLong_AsUnsignedLongLongMask(args[4]);
    if (PyErr_Occurred()) return -1;
    t->num_elem_allocated = t->num_elem;
    const long dtype = PyLong_AsLong(args[5]);
    if (dtype == -1 && PyErr_Occurred()) return -1;
    const long device = PyLong_AsLong(args[6]);
    if (device == -1 && PyErr_Occurred()) return -1;
    t->dtype = (int32_t)dtype;
    t->device_id = (int32_t)device;
    return 0;
}

/* bagua_comm_backend_mark_communication_ready_desc */
static PyObject* fp_backend_mark(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    void* h;
    const char* name;
    uint64_t ev;
    bagua_tensor_t t;
    (void)self;
    if (parse_mark(args, nargs, &h, &name, &ev, &t)) return NULL;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = bagua_comm_backend_mark_communication_ready_desc((BaguaCommBackendC*)h, name, ev, &t);
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

/* bagua_bucket_mark_tensor_ready_desc */
static PyObject* fp_bucket_mark(PyObject* self, PyObject* const* args, Py_ssize_t nargs) {
    void* h;
    const char* name;
    uint64_t ev;
    bagua_tensor_t t;
    (void)self;
    if (parse_mark(args, nargs, &h, &name, &ev, &t)) return NULL;
    int rc;
    Py_BEGIN_ALLOW_THREADS
    rc = bagua_bucket_mark_tensor_ready_desc((BaguaBucketC*)h, name, ev, &t);
    Py_END_ALLOW_THREADS
    return PyLong_FromLong(rc);
}

static PyMethodDef fp_methods[] = {
    {"backend_mark", (PyCFunction)(void (*)(void))fp_backend_mark, METH_FASTCALL,
     "backend_mark(handle, name, event, ptr, num_elem, dtype, device_id) -> status"},
    {"bucket_mark", (PyCFunction)(void (*)(void))fp_bucket_mark, METH_FASTCALL,
     "bucket_mark(handle, name, event, ptr, num_elem, dtype, device_id) -> status"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef fp_module = {PyModuleDef_HEAD_INIT, "_fastpath", NULL, -1, fp_methods,
                                       NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__fastpath(void) { return PyModule_Create(&fp_module); }
