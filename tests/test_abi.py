"""The C-ABI boundary: library loads and exports every symbol include/ygm.h declares
(no compute calls: this runs without a GPU)."""
import ctypes
import os
import re

from conftest import ROOT

import hocuspocus_amd.engine as eng


def header_functions():
    src = open(os.path.join(ROOT, "include", "ygm.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ygm_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    fns = header_functions()
    for f in ("ygm_merge_v1", "ygm_diff_v1", "ygm_sv_from_update_v1", "ygm_open", "ygm_close"):
        assert f in fns
    assert set(fns) == set(eng.EXPORTS)


def test_library_exports_every_declared_symbol():
    L = ctypes.CDLL(eng.LIB_PATH)
    for f in header_functions():
        assert hasattr(L, f), f


def test_strerror_and_version_without_gpu():
    assert "malformed" in eng.strerror(eng.EMALFORMED)
    assert eng.lib().ygm_version().startswith(b"ygm")


PRODUCT_DIRS = ("hocuspocus_amd", os.path.join("packages", "extension-gpu-merge", "src"),
                os.path.join("packages", "extension-gpu-merge", "addon"))


def test_no_cpu_fallback_in_product():
    # the product (Python package, Node extension and its N-API addon) never imports the oracle or the
    # test-only yjs bundle loader
    for d in PRODUCT_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            for f in fs:
                if f.endswith((".py", ".cpp", ".hip", ".hpp", ".h", ".js", ".cc", ".c")):
                    txt = open(os.path.join(dp, f), errors="ignore").read()
                    assert "import oracle" not in txt and "liboracle" not in txt, f
                    assert not re.search(r'#include\s*[<"][^">]*oracle', txt), f
                    assert not re.search(r"require\([^)]*(oracle|yjs_bundle)", txt), f


def test_gpumerge_reference_bytes_only_for_refused_documents():
    # GpuMerge stores the CPU Y.encodeStateAsUpdate(document) only for a per-document refusal; a failed
    # batch (EDEVICE / ENOMEM / a rejected native call) rethrows (device loss rejects the hook)
    src = open(os.path.join(ROOT, "packages", "extension-gpu-merge", "src", "index.js")).read()
    m = re.search(r"catch \(e\) \{(.*?)\n      \}", src[src.index("async onStoreDocument"):], flags=re.S)
    assert m, "onStoreDocument has its refusal handler"
    body = m.group(1)
    assert "if (!isRefusal(e) || " in body and body.index("isRefusal") < body.index("this._Y().encodeStateAsUpdate")
    refusals = re.search(r"REFUSALS = new Set\(\[(.*?)\]\)", src).group(1)
    for code in ("EDEVICE", "ENOMEM", "EINVAL"):
        assert code not in refusals
