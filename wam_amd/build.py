"""Build libwam_hip.so (gfx950) in-tree with hipcc.

    python -m wam_amd.build            # or: python wam_amd/build.py

No RPATH to /opt/rocm is recorded: the library binds to the libamdhip64.so.7 that torch has
already loaded (import torch before loading it; see wam_amd/_lib.py).
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libwam_hip.so")
SOURCES = ["plan.hip", "dwt_axis.hip", "dwt2_fused.hip", "dwt2_rows.hip", "dwt2_plane.hip", "dwt1_tile.hip", "dwt3_haar.hip", "epilogue.hip", "evaluate.hip", "visualize3d.hip", "melspec.hip", "model_ew.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("WAM_OFFLOAD_ARCH", "gfx950")


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "wam_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps)


def build(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    objs = []
    jobs = []
    for src in SOURCES:
        obj = os.path.join(CSRC, src.replace(".hip", ".o"))
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-c",
               "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics",
               os.path.join(CSRC, src), "-o", obj]
        objs.append(obj)
        jobs.append(subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    failed = False
    for src, j in zip(SOURCES, jobs):
        out, _ = j.communicate()
        if verbose or j.returncode:
            sys.stderr.write(out.decode())
        if j.returncode:
            failed = True
            sys.stderr.write("hipcc failed on %s\n" % src)
    if failed:
        raise RuntimeError("libwam_hip.so build failed")
    tmp = OUT + ".tmp"
    link = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.check_call(link)
    os.replace(tmp, OUT)
    for o in objs:
        os.remove(o)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
