"""Copy-engine probe from a Python process: does hipMemcpyDeviceToDeviceNoCU still go to the SDMA
engines once torch has initialised the GPU in the same process?  Run under
`rocprofv3 --kernel-trace --stats`: every copy the runtime turns into a blit kernel shows up as an
`__amd_rocclr_copyBuffer` dispatch (tools/copy_kind.py and tests/native/copy_kind_probe.cpp are
the native twins).  Phases, 20 copies each: NoCU 4-byte H2D, NoCU 56-byte D2H, then plain
hipMemcpyHostToDevice 4-byte H2D (a blit kernel on this runtime: the control).

  python3 tools/copy_kind_py.py <torch 0|1> [<host memory: hostmalloc|registered>]
"""
import ctypes as C
import importlib.util
import os
import sys

NOCU, H2D = 1024, 1  # hipMemcpyDeviceToDeviceNoCU, hipMemcpyHostToDevice


def main():
    use_torch = sys.argv[1] == "1"
    mem = sys.argv[2] if len(sys.argv) > 2 else "hostmalloc"
    if use_torch:
        import torch
        torch.zeros(1, device="cuda")
        torch.cuda.synchronize()
        tdir = os.path.dirname(torch.__file__)
    else:  # torch's runtime library without importing torch
        tdir = os.path.dirname(importlib.util.find_spec("torch").origin)
    hip = C.CDLL(os.path.join(tdir, "lib", "libamdhip64.so"))

    def ck(rc, what):
        if rc != 0:
            raise SystemExit(f"{what}: hip error {rc}")

    ck(hip.hipSetDevice(0), "hipSetDevice")
    st = C.c_void_p()
    ck(hip.hipStreamCreateWithFlags(C.byref(st), 1), "hipStreamCreateWithFlags")
    dev, hm = C.c_void_p(), C.c_void_p()
    ck(hip.hipMalloc(C.byref(dev), C.c_size_t(1 << 20)), "hipMalloc")
    if mem == "registered":
        buf = (C.c_char * (1 << 20))()
        hm = C.cast(buf, C.c_void_p)
        ck(hip.hipHostRegister(hm, C.c_size_t(1 << 20), 0), "hipHostRegister")
    else:
        ck(hip.hipHostMalloc(C.byref(hm), C.c_size_t(1 << 20), 0), "hipHostMalloc")
    cp = hip.hipMemcpyAsync
    cp.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    for n, dst, src, kind in ((4, dev, hm, NOCU), (56, hm, dev, NOCU), (4, dev, hm, H2D)):
        for _ in range(20):
            ck(cp(dst, src, n, kind, st), "hipMemcpyAsync")
        ck(hip.hipStreamSynchronize(st), "hipStreamSynchronize")
    print(f"copy_kind_py torch={int(use_torch)} mem={mem}: 60 copies issued "
          "(20 of them blit kernels expected if NoCU stays on SDMA)")


if __name__ == "__main__":
    main()
