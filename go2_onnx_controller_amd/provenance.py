"""Which kernel sources a committed profile was taken from.

bench.py reports roofline.traffic from the committed rocprofv3 --pmc summary
(profiles/pmc_summary.json) rather than collecting counters in the timed run (a
--pmc pass is its own process). A summary entry carries the digest of the kernel
sources it was measured on; when the sources have changed since, the entry no
longer describes the kernel the bench runs, and bench.py reports traffic as null
with the reason instead of a stale number."""
import glob
import hashlib
import os

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "csrc")


def kernel_source_digest() -> str:
    """sha256 (first 16 hex) over every source that decides what the device runs and
    the build flags: csrc/*.hip, *.hpp, *.inc (the kernels), engine.cpp and
    onnx_model.cpp (weight packing and padding, kernel choice and launch shapes: a
    packing change moves the traffic as surely as a kernel change) and the
    Makefile, in name order."""
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(CSRC, "*.hip")) + glob.glob(os.path.join(CSRC, "*.hpp")) +
                   glob.glob(os.path.join(CSRC, "*.inc")) + glob.glob(os.path.join(CSRC, "*.cpp")) +
                   [os.path.join(CSRC, "Makefile")])
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
