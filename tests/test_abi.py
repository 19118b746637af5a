"""CPU: the C-ABI library loads, exports every symbol include/capgen.h declares, and its
host-only parameter table matches the reference state_dict (no device calls)."""
import os
import re

import pytest

from capgen import _lib, preset
from capgen.params import reference_param_specs, num_params

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(REPO, "include", "capgen.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(capgen_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    declared = header_functions()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert sorted(_lib.EXPORTED) == declared


def test_abi_version():
    assert _lib.load().capgen_abi_version() == _lib.ABI_VERSION


VARIANTS = {"plain": {}, "imgobj": {"split_image_objects": True}, "movefirst": {"move_first_image_feature": True},
            "both": {"split_image_objects": True, "move_first_image_feature": True}}


@pytest.mark.parametrize("variant", sorted(VARIANTS))
@pytest.mark.parametrize("name", ["C1", "C2"])
def test_param_table_matches_reference_specs(name, variant):
    cfg = preset(name, **VARIANTS[variant])
    table, total = _lib.param_table(cfg)
    specs = reference_param_specs(cfg)
    assert [t[0] for t in table] == [s[0] for s in specs]
    covered = 0
    spans = []
    for (n, ndim, rows, cols, off, stride), (_, shape) in zip(table, specs):
        assert ndim == len(shape)
        assert (rows, cols) == (shape if ndim == 2 else (1, shape[0]))
        assert stride >= cols
        spans.append((off, off + (rows - 1) * stride + cols, n))
        covered += rows * cols
    assert covered == num_params(cfg)
    if variant == "plain":
        assert covered == (55707408 if name == "C2" else 1272808)
    # no two tensors overlap (interleaved strided tensors checked element-wise below)
    occ = bytearray(total)
    for (n, ndim, rows, cols, off, stride) in table:
        for r in range(rows):
            seg = occ[off + r * stride: off + r * stride + cols]
            assert not any(seg), n
            occ[off + r * stride: off + r * stride + cols] = b"\x01" * cols
    assert max(s[1] for s in spans) <= total


def test_bad_config_raises_loudly():
    cfg = preset("C1", num_vocab=1001)
    with pytest.raises(NotImplementedError):
        _lib.param_table(cfg)
    cfg = preset("C1", split_image_objects=True, split_position=True)  # fails in the reference too
    with pytest.raises(NotImplementedError):
        _lib.param_table(cfg)


def test_split_position_names_the_same_columns():
    """SPLIT_POSITION (model.py:231-233, 297-303): object_embedding [d, P-4] then
    position_embedding [d, 4], together exactly the unsplit position columns."""
    plain, n0 = _lib.param_table(preset("C1"))
    split, n1 = _lib.param_table(preset("C1", split_position=True))
    assert n0 == n1
    t0 = {e[0]: e for e in plain}
    t1 = {e[0]: e for e in split}
    assert [e[0] for e in split][:2] == ["encoder.object_embedding.weight", "encoder.position_embedding.weight"]
    _, _, rows, cols, off, stride = t0["encoder.position_embedding.weight"]
    o = t1["encoder.object_embedding.weight"]
    p = t1["encoder.position_embedding.weight"]
    assert (p[2], p[3], p[4], p[5]) == (rows, 4, off, stride)
    assert (o[2], o[3], o[4], o[5]) == (rows, cols - 4, off + 4, stride)
    assert {k: v for k, v in t0.items() if "position_embedding" not in k} == \
        {k: v for k, v in t1.items() if "_embedding.weight" not in k or "feature" in k or "word" in k}


def test_engine_refuses_cpu_device():
    from capgen.engine import Engine
    with pytest.raises(RuntimeError):
        Engine(preset("C1"), "cpu")
