"""Build libwam_hip.so (gfx950) in-tree with hipcc.

    python wam_amd/build.py            # or: python -m wam_amd.build

No RPATH to /opt/rocm is recorded: the library binds to the libamdhip64.so.7 that torch has
already loaded (import torch before loading it; see wam_amd/_lib.py).

Objects are cached under build/obj/ by a hash of their source, the shared headers and the compile
line, so a build after a one-file change (and the variant builds of scripts/build_variants.py)
recompiles that file only.
"""
import functools
import hashlib
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
OUT = os.path.join(HERE, "libwam_hip.so")
OBJ_CACHE = os.path.join(os.path.dirname(HERE), "build", "obj")
SOURCES = ["plan.hip", "dwt_axis.hip", "dwt2_fused.hip", "dwt2_rows.hip", "dwt2_plane.hip",
           "dwt1_tile.hip", "dwt3_haar.hip", "dwt3_tile.hip", "epilogue.hip", "evaluate.hip", "visualize3d.hip", "melspec.hip",
           "model_ew.hip"]
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("WAM_OFFLOAD_ARCH", "gfx950")


def _stale():
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    deps = [os.path.join(CSRC, f) for f in os.listdir(CSRC)]
    deps.append(os.path.join(os.path.dirname(HERE), "include", "wam_hip.h"))
    return any(os.path.getmtime(d) > t for d in deps)


@functools.lru_cache(None)
def _toolchain():
    """hipcc's version banner and the HIPCC_* environment: a ROCm upgrade or a changed compile
    environment must not link objects from the old one."""
    try:
        ver = subprocess.run([HIPCC, "--version"], stdout=subprocess.PIPE, stderr=subprocess.STDOUT).stdout
    except OSError:
        ver = b"?"
    env = "".join("%s=%s;" % kv for kv in sorted(os.environ.items()) if kv[0].startswith("HIPCC_"))
    return ver + env.encode()


def _key(src, cmd):
    h = hashlib.sha1(" ".join(cmd[:-3]).encode())
    h.update(_toolchain())
    hdrs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hpp"))
    for f in [src] + [os.path.join(CSRC, x) for x in hdrs] + [os.path.join(CSRC, "..", "..", "include", "wam_hip.h")]:
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def build(force=False, verbose=False):
    if not force and not _stale():
        return OUT
    os.makedirs(OBJ_CACHE, exist_ok=True)
    objs = []
    jobs = []
    for src in SOURCES:
        path = os.path.join(CSRC, src)
        # a unique temporary object per process, moved into the cache atomically (concurrent builds)
        fd, tmp_obj = tempfile.mkstemp(suffix=".o", prefix=src.replace(".hip", "."), dir=OBJ_CACHE)
        os.close(fd)
        cmd = [HIPCC, "--offload-arch=" + ARCH, "-O3", "-std=c++17", "-fPIC", "-c",
               "-Wall", "-Wno-unused-function", "-munsafe-fp-atomics", path, "-o", tmp_obj]
        cached = os.path.join(OBJ_CACHE, "%s.%s.o" % (src, _key(path, cmd)))
        objs.append(cached)
        if os.path.exists(cached):
            os.unlink(tmp_obj)
            continue
        jobs.append((src, tmp_obj, cached, subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)))
    failed = False
    for src, tmp_obj, cached, j in jobs:
        out, _ = j.communicate()
        if verbose or j.returncode:
            sys.stderr.write(out.decode())
        if j.returncode:
            failed = True
            sys.stderr.write("hipcc failed on %s\n" % src)
            if os.path.exists(tmp_obj):
                os.unlink(tmp_obj)
        else:
            os.replace(tmp_obj, cached)
    if failed:
        raise RuntimeError("libwam_hip.so build failed")
    tmp = "%s.%d.tmp" % (OUT, os.getpid())
    link = [HIPCC, "--offload-arch=" + ARCH, "-shared", "-fPIC", "-o", tmp] + objs
    subprocess.check_call(link)
    os.replace(tmp, OUT)
    return OUT


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose="-v" in sys.argv))
