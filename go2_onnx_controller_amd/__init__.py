"""go2pi — MI355X-native batched policy inference behind the reference's
`ONNXActor::act()` boundary (inria-paris-robotics-lab/go2_onnx_controller,
onnx_inference/include/onnx_actor.hpp).

Product path: libgo2pi.so (HIP kernels for gfx950 + C ABI, include/go2pi.h)
and libonnx_actor.so (drop-in C++ ONNXActor, include/onnx_actor.hpp). This
package adds the Python mirrors (`ONNXActor`, `InferenceSession`), the ctypes
`Engine`, the deterministic synthetic policies and the many-robot sharding.
"""
from .engine import Engine, Go2piError, LIB_PATH, ACTOR_LIB_PATH  # noqa: F401
from .actor import ONNXActor, InferenceSession  # noqa: F401

__version__ = "0.1.0"
