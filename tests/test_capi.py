"""The C-ABI library loads and exports every symbol include/wam_hip.h declares (CPU; no compute)."""
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "wam_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(wam_[a-z0-9_]+)\s*\(", src)))


def test_header_symbols_exported_and_bound():
    from wam_amd import _lib
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(_lib.lib, n), "libwam_hip.so does not export %s" % n
        assert n in _lib._SIGS, "%s declared in the header but not bound in wam_amd/_lib.py" % n
    assert set(_lib._SIGS) == set(names)


def test_host_only_entry_points():
    from wam_amd import _lib
    assert _lib.lib.wam_version() == 2
    assert b"shape" in _lib.lib.wam_strerror(2)
    assert _lib.lib.wam_strerror(0) == b"success"
    # NULL plan arguments are rejected without touching the device
    assert _lib.lib.wam_plan_num_bands(None) < 0
    assert _lib.lib.wam_wavedec(None, 1, None, None, None, None) == 1


def test_gfx950_code_object():
    blob = open(os.path.join(REPO, "wam_amd", "libwam_hip.so"), "rb").read()
    assert b"gfx950" in blob


def test_import_fails_loudly_without_library(tmp_path):
    """No silent fallback: importing the package without libwam_hip.so raises ImportError."""
    import shutil
    dst = tmp_path / "wam_amd"
    shutil.copytree(os.path.join(REPO, "wam_amd"), dst, ignore=shutil.ignore_patterns("*.so", "__pycache__"))
    code = "import sys; sys.path.insert(0, %r); import wam_amd" % str(tmp_path)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True)
    assert r.returncode != 0 and "libwam_hip.so" in r.stderr and "ImportError" in r.stderr
