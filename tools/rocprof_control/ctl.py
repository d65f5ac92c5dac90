"""rocprofv3 exit-crash control: a Python process that runs one HIP kernel through ctypes
(libcontrol.so, no libfisdf) — with ``--torch`` through torch instead.  argv[1]: where to write
/proc/self/maps (to symbolize a crash in the exit handlers)."""
import ctypes
import os
import sys


def main():
    if "--torch" in sys.argv:
        import torch
        x = torch.ones(1 << 20, dtype=torch.float64, device="cuda")
        for _ in range(10):
            x.mul_(2.0)
        torch.cuda.synchronize()
        print("torch control ok", float(x[0]))
    else:
        lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libcontrol.so"))
        print("control_run rc =", lib.control_run(1 << 20))
    with open("/proc/self/maps") as src, open(sys.argv[1], "w") as dst:
        dst.write(src.read())


if __name__ == "__main__":
    main()
