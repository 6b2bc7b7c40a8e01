"""Device buffers for GPU tests through the HIP runtime libslam_ekf.so itself links
(libamdhip64.so.7), not torch: torch bundles its own HIP runtime, and whichever of the two
initialises second in a process may find no device."""
import ctypes

import numpy as np

_hip = None


def hip():
    global _hip
    if _hip is None:
        from slam_ros_amd import ekf
        ekf.load_library()                       # loads libamdhip64.so.7 as its dependency
        _hip = ctypes.CDLL("libamdhip64.so.7")
        _hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
        _hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _hip.hipFree.argtypes = [ctypes.c_void_p]
    return _hip


class DeviceArray:
    """A host array copied to device memory (freed on close)."""

    def __init__(self, host: np.ndarray):
        host = np.ascontiguousarray(host)
        self.nbytes = host.nbytes
        self.ptr = ctypes.c_void_p()
        assert hip().hipMalloc(ctypes.byref(self.ptr), self.nbytes) == 0, "hipMalloc"
        assert hip().hipMemcpy(self.ptr, host.ctypes.data_as(ctypes.c_void_p), self.nbytes, 1) == 0, "hipMemcpy"

    @property
    def address(self) -> int:
        return int(self.ptr.value)

    def close(self):
        if self.ptr:
            hip().hipFree(self.ptr)
            self.ptr = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def gpu_present() -> bool:
    """hipGetDeviceCount through the library's own HIP runtime (no torch)."""
    try:
        n = ctypes.c_int(0)
        return hip().hipGetDeviceCount(ctypes.byref(n)) == 0 and n.value > 0
    except OSError:
        return False
