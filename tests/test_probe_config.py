"""CPU: the obliviousness test's shapes name only mixes the probe defines
(tests/test_oblivious.py SHAPES against tools/oblivious_probe.py MIXES and
KV_MIXES), so a renamed mix cannot silently drop out of the GPU counter run."""
import importlib.util
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(name, path):
    spec = importlib.util.spec_from_file_location(name, path)
    mod = importlib.util.module_from_spec(spec)
    sys.modules[name] = mod
    spec.loader.exec_module(mod)
    return mod


def test_shapes_use_probe_mixes():
    probe = load("oblivious_probe", os.path.join(ROOT, "tools", "oblivious_probe.py"))
    obl = load("test_oblivious_shapes", os.path.join(ROOT, "tests", "test_oblivious.py"))
    for shape, spec in obl.SHAPES.items():
        args = spec["args"]
        kind = "oram" if "--oram" in args else "omap" if "--omap" in args else None
        known = set(probe.KV_MIXES[kind]) if kind else set(probe.MIXES)
        assert "main" in spec["mixes"], shape  # the reference every mix is compared with
        for mix in list(spec["mixes"]) + list(spec.get("pmc_mixes", [])):
            assert mix in known, (shape, mix)
        if not kind and "--wire" not in args:
            assert not any(m.startswith("wire_") for m in spec["mixes"]), shape


def test_kv_mix_parameters():
    probe = load("oblivious_probe", os.path.join(ROOT, "tools", "oblivious_probe.py"))
    for pool, p in probe.KV_MIXES["oram"].values():
        assert pool in ("uniform", "hot", "one") and 0.0 <= p <= 1.0
    for pool, p in probe.KV_MIXES["omap"].values():
        assert pool in ("uniform", "hot", "fresh") and len(p) == 4 and abs(sum(p) - 1.0) < 1e-9


def test_expiry_and_timing_shapes():
    """x_* mixes only with --expiry; the timing shapes name probe mixes, and
    the expiry cutoffs expire nothing, everything, or a few rows."""
    probe = load("oblivious_probe", os.path.join(ROOT, "tools", "oblivious_probe.py"))
    obl = load("test_oblivious_shapes", os.path.join(ROOT, "tests", "test_oblivious.py"))
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    tim = load("test_timing_shapes", os.path.join(ROOT, "tests", "test_timing.py"))
    for shapes in (obl.SHAPES, tim.SHAPES):
        for shape, spec in shapes.items():
            if "--oram" in spec["args"] or "--omap" in spec["args"]:
                continue  # KV mixes: test_shapes_use_probe_mixes
            x = "--expiry" in spec["args"]
            for mix in spec["mixes"]:
                assert mix in probe.MIXES, (shape, mix)
                assert mix.startswith("x_") == (x and mix != "main"), (shape, mix)
    for k in range(6):
        assert probe.expiry_cutoff("x_none", k) == 0
        assert probe.expiry_cutoff("x_all", k) > probe.TS0 + 10**9
        assert probe.expiry_cutoff("x_few", k) == probe.TS0 + 1 + 16 * (k + 1)
    for spec in tim.SHAPES.values():
        assert spec["ref"] in spec["mixes"]
