"""Which allocation calls HIP permits on a non-capturing stream while another stream of the process
captures a graph in global mode (torch.cuda.graph's default): plain hipMalloc, hipMalloc with this
thread switched to relaxed capture mode, hipMallocAsync on the side stream. Prints return codes only."""
import ctypes

import torch

hip = ctypes.CDLL("libamdhip64.so")
hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
hip.hipMallocAsync.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_void_p]
hip.hipThreadExchangeStreamCaptureMode.argtypes = [ctypes.POINTER(ctypes.c_int)]
hip.hipGetLastError.restype = ctypes.c_int


def attempt(kind, side):
    p = ctypes.c_void_p()
    x = torch.zeros(16, device="cuda")
    g = torch.cuda.CUDAGraph()
    res = {}
    try:
        with torch.cuda.graph(g):
            y = x * 2  # noqa: F841
            if kind == "plain":
                res["rc"] = hip.hipMalloc(ctypes.byref(p), 1 << 20)
            elif kind == "relaxed":
                mode = ctypes.c_int(2)  # hipStreamCaptureModeRelaxed
                res["xchg"] = hip.hipThreadExchangeStreamCaptureMode(ctypes.byref(mode))
                res["rc"] = hip.hipMalloc(ctypes.byref(p), 1 << 20)
                res["xchg_back"] = hip.hipThreadExchangeStreamCaptureMode(ctypes.byref(mode))
                res["prev_mode"] = mode.value
            elif kind == "async":
                res["rc"] = hip.hipMallocAsync(ctypes.byref(p), 1 << 20, ctypes.c_void_p(side.cuda_stream))
            res["last_err"] = hip.hipGetLastError()
        g.replay()
        torch.cuda.synchronize()
        res["capture"] = "ok"
    except Exception as e:  # noqa: BLE001
        res["capture"] = f"failed: {str(e).splitlines()[0]}"
        hip.hipGetLastError()
    print(kind, res, flush=True)


side = torch.cuda.Stream()
for kind in ("relaxed", "async", "plain"):
    attempt(kind, side)
