#!/usr/bin/env python3
"""A/B probe (GPU box): the bench frame with the render side stream created
under a CU mask (hipExtStreamCreateWithCUMask), so that the global photon
trace's launches on the main stream always find free CUs beside the render's
pool kernels. Runs bench.py's main in-process with GpuBackend's side stream
replaced; prints the bench line.
    python tools/cumask_probe.py MASKWORD -- bench args
MASKWORD: a 32-bit pattern repeated over the CU mask words (e.g. 0x77777777 =
3 of every 4 CUs); "none" leaves the stream as it is."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "photon-mapping_amd")]


def main():
    word = sys.argv[1]
    rest = sys.argv[sys.argv.index("--") + 1:] if "--" in sys.argv else []
    import torch
    from pm_amd import dist as pmdist
    if word != "none":
        hip = ctypes.CDLL("libamdhip64.so.7")
        fn = hip.hipExtStreamCreateWithCUMask
        fn.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32)]
        fn.restype = ctypes.c_int
        ncu = torch.cuda.get_device_properties(0).multi_processor_count
        nw = (ncu + 31) // 32
        mask = (ctypes.c_uint32 * nw)(*([int(word, 16)] * nw))
        orig = pmdist.GpuBackend.__init__

        def init(self, *a, **k):
            orig(self, *a, **k)
            h = ctypes.c_void_p()
            st = fn(ctypes.byref(h), nw, mask)
            if st != 0:
                raise RuntimeError(f"hipExtStreamCreateWithCUMask: {st}")
            self._rside = torch.cuda.ExternalStream(h.value)
            print(f"side stream CU mask {word} x {nw} words ({ncu} CUs)", file=sys.stderr, flush=True)

        pmdist.GpuBackend.__init__ = init
    import bench
    sys.argv = ["bench.py"] + rest
    bench.main()


if __name__ == "__main__":
    main()
