"""CPU-side checks of the C-ABI library: it loads and exports every symbol the header declares
(no compute calls — there is no GPU here)."""
import ctypes
import os
import re

import pytest

from .conftest import ROOT

HEADER = os.path.join(ROOT, "include", "autovc_hip.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(avc_[a-z0-9_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from autoformer_amd import _lib

    if not os.path.exists(_lib.LIB_PATH):
        _lib.build()
    return _lib.lib()


def test_header_declares_entry_points():
    syms = declared_symbols()
    assert "avc_gemm" in syms and "avc_lstm_fwd" in syms and len(syms) >= 25


def test_library_exports_every_declared_symbol(lib):
    so = ctypes.CDLL(os.path.join(ROOT, "autoformer_amd", "libautovc_hip.so"))
    missing = [s for s in declared_symbols() if not hasattr(so, s)]
    assert not missing, missing


def test_python_binding_covers_header(lib):
    from autoformer_amd import _lib

    assert set(_lib.exported_symbols()) == set(declared_symbols())


def test_abi_version_and_error_channel(lib):
    assert lib.avc_abi_version() == 31
    assert isinstance(lib.avc_last_error(), bytes)


def test_argument_validation_without_gpu(lib):
    from autoformer_amd import _lib

    # null descriptor is rejected on the host before any launch
    rc = lib.avc_gemm(None, None)
    assert rc != 0
    assert b"null" in lib.avc_last_error()
    with pytest.raises(RuntimeError):
        _lib.check(rc, "avc_gemm")


def test_struct_layout_matches_header(tmp_path):
    """Field offsets of the ctypes structs == what a C compiler makes of include/autovc_hip.h."""
    import subprocess

    from autoformer_amd import _lib

    fields = {"avc_operand": [f[0] for f in _lib.Operand._fields_], "avc_gemm_desc": [f[0] for f in _lib.GemmDesc._fields_],
              "avc_pack_op": [f[0] for f in _lib.PackOp._fields_], "avc_bn_fin": [f[0] for f in _lib.BnFin._fields_]}
    src = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){"]
    for st, fs in fields.items():
        src.append(f'printf("{st} %zu\\n", sizeof({st}));')
        for f in fs:
            src.append(f'printf("{st}.{f} %zu\\n", offsetof({st}, {f}));')
    src.append("return 0;}")
    c = tmp_path / "probe.c"
    c.write_text("\n".join(src))
    exe = tmp_path / "probe"
    subprocess.run(["gcc", str(c), "-o", str(exe)], check=True)
    out = dict(line.rsplit(" ", 1) for line in subprocess.run([str(exe)], capture_output=True, text=True,
                                                               check=True).stdout.split("\n") if line)
    for st, cls in (("avc_operand", _lib.Operand), ("avc_gemm_desc", _lib.GemmDesc), ("avc_pack_op", _lib.PackOp),
                    ("avc_bn_fin", _lib.BnFin)):
        assert int(out[st]) == ctypes.sizeof(cls), st
        for f in fields[st]:
            assert int(out[f"{st}.{f}"]) == getattr(cls, f).offset, (st, f)


def test_product_path_does_not_import_oracle():
    for dirpath, _, files in os.walk(os.path.join(ROOT, "autoformer_amd")):
        for f in files:
            if f.endswith(".py"):
                txt = open(os.path.join(dirpath, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt, f


def test_factory_state_dict_layout_matches_reference():
    import json

    import factory.AutoVC as A

    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "state_dict_layout.json")))
    m = A.AutoVC(44, 256, 512, 22)
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == ref["AutoVC"]


def test_ops_refuse_cpu_tensors(lib):
    import torch

    import factory.AutoVC as A

    m = A.AutoVC(44, 256, 512, 22)
    with pytest.raises(RuntimeError):
        m(torch.zeros(2, 176, 80), torch.zeros(2, 256), torch.zeros(2, 256))


@pytest.mark.parametrize("mod,cls", [("factory.MetaConv", "MetaConv"), ("factory.MetaPool", "MetaPool")])
def test_metaformer_state_dict_layout_matches_reference(mod, cls):
    import importlib
    import json

    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "state_dict_layout.json")))
    m = getattr(importlib.import_module(mod), cls)(44, 256, 512, 22)
    assert [[k, list(v.shape)] for k, v in m.state_dict().items()] == ref[cls]


def test_counter_ring_reservations_never_overlap(lib):
    """the slot ring behind the split-K / BN arrival counters must hand out
    disjoint ranges across its wrap (a crossing request restarts at 0 and the cursor moves past it)."""
    import random

    pool = 1 << 10
    cur = ctypes.c_uint(0)
    rng = random.Random(7)
    live = []  # the last reservations, fewer than `pool` slots in total
    for i in range(5000):
        n = rng.choice([1, 3, 16, 64, 200, 256, 511])
        b = lib.avc_ring_reserve_test(ctypes.byref(cur), n, pool)
        assert 0 <= b and b + n <= pool, (i, b, n)
        live.append((b, n))
        while sum(m for _, m in live) > pool // 2:
            live.pop(0)
        for b2, n2 in live[:-1]:
            assert b + n <= b2 or b2 + n2 <= b, (i, (b, n), (b2, n2))
    # the cursor also wraps modulo 2^32 cleanly (pool divides 2^32)
    cur = ctypes.c_uint(0xFFFFFFFF - 5)
    b = lib.avc_ring_reserve_test(ctypes.byref(cur), 16, pool)
    assert b == 0 and lib.avc_ring_reserve_test(ctypes.byref(cur), 4, pool) == 16
