"""The committed golden fixtures (tests/golden/) against the CPU restatement:
the oracle must still reproduce them byte for byte (a change to the oracle's
semantics shows up here first).  The GPU engine is checked against the same
files in tests/test_gpu_parity.py::test_golden_fixtures."""
import hashlib
import json
import os

import pytest

from oracle import ffi

from golden_io import GOLDEN, NAMES, load


def test_manifest_hashes():
    man = json.load(open(os.path.join(GOLDEN, "MANIFEST.json")))
    assert set(man) == {n + ".npz" for n in NAMES}
    for f, h in man.items():
        assert hashlib.sha256(open(os.path.join(GOLDEN, f), "rb").read()).hexdigest() == h, f


@pytest.mark.parametrize("name", NAMES)
def test_oracle_reproduces_golden(name):
    cfg, batches = load(name)
    model = ffi.Cluster(cfg) if cfg.shard_count > 1 else ffi.Model(cfg)
    for k, (reqs, want, (msgs, mboxes)) in enumerate(batches):
        got = model.process_batch(reqs)
        assert got.tobytes() == want.tobytes(), (name, k)
        assert (model.messages, model.mailboxes) == (msgs, mboxes), (name, k)


def test_golden_covers_every_status():
    seen = set()
    for name in NAMES:
        for _, resp, _ in load(name)[1]:
            seen.update(int(s) for s in resp["status_code"])
    assert {0, 1, 2, 4, 5, 6, 7} <= seen, seen
