"""Build tools/bin/convbench: the engine's kernel sources (with their per-file flags from build.py)
plus the knock-out / variant launchers (-DCLASFV_KNOCKOUTS) and tools/convbench.hip. Not product."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
import clasfv_amd.build as B  # noqa: E402

KERNELS = ["winograd.hip", "winograd2.hip", "winograd4.hip", "winograd4w.hip", "winograd_t.hip", "conv.hip", "conv_patch.hip", "decoder.hip",
           "twalk.hip"]
# measured-slower design points kept out of the product library
EXPERIMENTAL = ["winograd3.hip", "winograd_w.hip", "winograd_s.hip"]


def main():
    out = os.path.join(HERE, "bin")
    os.makedirs(os.path.join(out, "obj"), exist_ok=True)
    hipcc = B._hipcc()
    flags = [f"--offload-arch={B.ARCH}", "-O3", "-std=c++17", "-DCLASFV_KNOCKOUTS", "-I", B.INCLUDE, "-I", B.CSRC]
    jobs = [(os.path.join(B.CSRC, f), B.EXTRA_FLAGS.get(f, [])) for f in KERNELS]
    jobs += [(os.path.join(HERE, "experimental", f), []) for f in EXPERIMENTAL]
    jobs.append((os.path.join(HERE, "convbench.hip"), []))
    jobs.append((os.path.join(HERE, "conv_patch_v1.hip"), []))
    jobs.append((os.path.join(HERE, "winoq_probe.hip"), []))

    def cc(job):
        src, extra = job
        obj = os.path.join(out, "obj", os.path.basename(src) + ".o")
        r = subprocess.run([hipcc] + flags + extra + ["-c", src, "-o", obj], capture_output=True, text=True)
        if r.returncode:
            raise RuntimeError(r.stderr[-4000:])
        return obj

    with ThreadPoolExecutor(8) as ex:
        objs = list(ex.map(cc, jobs))
    subprocess.run([hipcc, f"--offload-arch={B.ARCH}", "-o", os.path.join(out, "convbench")] + objs, check=True)
    print(os.path.join(out, "convbench"))


if __name__ == "__main__":
    main()
