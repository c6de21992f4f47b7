"""Build experimental variants of libwam_hip.so into build/exp/<name>.so (git-ignored; they travel
to the GPU box with the tree) from the in-tree sources plus text substitutions, for A/B kernel
timing with WAM_LIB_PATH=build/exp/<name>.so python scripts/kbench.py.

usage: python scripts/build_variants.py <name>=<file>:<old>=><new>[||<file>:<old>=><new>] ...
       a part of the form <file>@<git-rev> takes that file from a git revision instead.
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    from wam_amd import build as B
    out_dir = os.path.join(REPO, "build", "exp")
    os.makedirs(out_dir, exist_ok=True)
    for spec in sys.argv[1:]:
        name, _, edits = spec.partition("=")
        tmp = tempfile.mkdtemp()
        src = os.path.join(tmp, "wam_amd", "csrc")
        shutil.copytree(os.path.join(REPO, "wam_amd", "csrc"), src)
        shutil.copytree(os.path.join(REPO, "include"), os.path.join(tmp, "include"))
        for e in filter(None, edits.split("||")):
            if "@" in e and "=>" not in e:
                f, rev = e.split("@")
                txt = subprocess.check_output(["git", "-C", REPO, "show", "%s:wam_amd/csrc/%s" % (rev, f)]).decode()
                open(os.path.join(src, f), "w").write(txt)
                continue
            f, _, rest = e.partition(":")
            old, new = rest.split("=>")
            p = os.path.join(src, f)
            t = open(p).read()
            assert old in t, (name, f, old)
            open(p, "w").write(t.replace(old, new))
        B.CSRC, B.OUT = src, os.path.join(out_dir, name + ".so")
        B.build(force=True)
        shutil.rmtree(tmp)
        print("built", B.OUT)


if __name__ == "__main__":
    main()
