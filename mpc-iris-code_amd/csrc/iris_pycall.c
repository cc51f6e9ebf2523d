/* iris_pycall.c -- the Python mirror's per-call fast path (CPython extension _iris_pycall).
 *
 * The reference's participant and resolver call batch_process(out, chunk) once per 20 000-record
 * slice (src/main.rs:426-431, 511-516); from Python through ctypes each call paid ~3.5 us of
 * binding (two numpy .ctypes.data lookups at ~1.3-1.8 us each, the foreign call itself) against
 * ~12.6 us of library work for a masks chunk from C++ (profiles/r06l_bench_host-masks_mmap.jsonl,
 * cxx_walk).  This module takes the two arrays through the buffer protocol and calls
 * iris_engine_batch_process_host with the GIL released; it adds no logic of its own.  Built beside
 * libiris_hip.so (Makefile) and linked to it; iris_hip.py uses it when present, ctypes otherwise. */
#define PY_SSIZE_T_CLEAN
#include <Python.h>

#include "../../include/iris_hip.h"

/* batch_process_host(engine: int, records, out, rec_bytes: int) -> int status
 * records: C-contiguous buffer of n whole records of rec_bytes; out: writable C-contiguous buffer of
 * n * 31 uint16.  A length mismatch returns IRIS_E_ARG with iris_last_error() unset (the caller
 * raises the reference's assertion message). */
static PyObject *batch_process_host(PyObject *self, PyObject *args) {
    unsigned long long engine = 0;
    PyObject *recs = NULL, *out = NULL;
    Py_ssize_t rec_bytes = 0;
    (void)self;
    if (!PyArg_ParseTuple(args, "KOOn", &engine, &recs, &out, &rec_bytes)) return NULL;
    if (rec_bytes <= 0) return PyLong_FromLong(IRIS_E_ARG);
    Py_buffer rv, ov;
    if (PyObject_GetBuffer(recs, &rv, PyBUF_C_CONTIGUOUS) != 0) return NULL;
    if (PyObject_GetBuffer(out, &ov, PyBUF_C_CONTIGUOUS | PyBUF_WRITABLE) != 0) {
        PyBuffer_Release(&rv);
        return NULL;
    }
    int rc = IRIS_E_ARG;
    const Py_ssize_t n = rv.len / rec_bytes;
    if (rv.len % rec_bytes == 0 && ov.len == n * (Py_ssize_t)(IRIS_ROTATIONS * sizeof(uint16_t))) {
        Py_BEGIN_ALLOW_THREADS
        rc = iris_engine_batch_process_host((iris_engine_t *)(uintptr_t)engine, rv.buf, (uint64_t)n, (uint16_t *)ov.buf);
        Py_END_ALLOW_THREADS
    }
    PyBuffer_Release(&ov);
    PyBuffer_Release(&rv);
    return PyLong_FromLong(rc);
}

static PyMethodDef methods[] = {
    {"batch_process_host", batch_process_host, METH_VARARGS, "iris_engine_batch_process_host over two buffers"},
    {NULL, NULL, 0, NULL},
};

static struct PyModuleDef module = {PyModuleDef_HEAD_INIT, "_iris_pycall", NULL, -1, methods, NULL, NULL, NULL, NULL};

PyMODINIT_FUNC PyInit__iris_pycall(void) { return PyModule_Create(&module); }
