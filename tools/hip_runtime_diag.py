import ctypes, sys
sys.path[:0] = ["mpc-iris-code_amd", "."]
import iris_hip as ih
print("pycall", ih._pycall is not None)
import torch.distributed  # noqa
dev = ih.Device(0)
def maps():
    return sorted({l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l})
print("mapped after open:", maps())
for name in ("libamdhip64.so", "libamdhip64.so.7"):
    h = ctypes.CDLL(name)
    n = ctypes.c_int()
    print(name, "hipGetDeviceCount rc", h.hipGetDeviceCount(ctypes.byref(n)), n.value)
    p = ctypes.c_void_p()
    h.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    print(name, "hipMalloc rc", h.hipMalloc(ctypes.byref(p), 1 << 20))
print("mapped at end:", maps())
