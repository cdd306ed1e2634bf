"""The counter harness's environment rules on synthetic per-batch data (CPU):
the one-batch re-walk exclusion and the re-measured whole-process re-walk
(tests/test_oblivious.py exclusions(), rewalk_processes())."""
import test_oblivious as ob


def _proc(ucs):
    # one kernel per batch: (kernel, grid, workgroup, value, uncached requests)
    return [[("k", 1, 1, 100.0, float(u))] for u in ucs]


def _pre(x):
    return [4000.0, 3900.0, 3800.0] + x  # 3 prefill batches (first touch walks)


def test_one_rewalk_batch_is_set_aside():
    per = {"main": _proc(_pre([10] * ob.N_MEAS)),
           "rud": _proc(_pre([10, 10, 2500, 10, 10, 10])),
           "main#2": _proc(_pre([10] * ob.N_MEAS))}
    ex = ob.exclusions(per)
    assert ex["rud"] == {5} and not ex["main"] and not ex["main#2"]


def test_two_rewalk_batches_are_kept():
    per = {"main": _proc(_pre([10] * ob.N_MEAS)),
           "rud": _proc(_pre([2500, 10, 2500, 10, 10, 10])),
           "main#2": _proc(_pre([10] * ob.N_MEAS))}
    assert not ob.exclusions(per)["rud"]


def test_whole_process_rewalk_is_measured_again():
    quiet = _proc(_pre([20, 60, 30, 10, 40, 20]))
    per = {"main": quiet, "rud": quiet, "deletes": _proc(_pre([310, 416, 342, 348, 358, 435])),
           "hot_next": quiet, "main#2": quiet}
    assert ob.rewalk_processes(per) == ["deletes"]
    # within 3x of the shape's median: no re-run
    per["deletes"] = _proc(_pre([50, 55, 60, 45, 70, 55]))
    assert ob.rewalk_processes(per) == []


# ---- the timing test's rules (tests/test_timing.py evaluate(), evaluate_interleaved())

import random  # noqa: E402

import test_timing as tt  # noqa: E402

KERNELS = [("k_sort", 5.0), ("k_scan", 6.0), ("k_pass", 5600.0)]


def _timing_proc(seed, n_batches=3 + tt.N_MEAS, bump=None, scale=1.0):
    """One process: per-batch (kernel, us) with small noise; bump = {(measured
    batch, kernel index): extra us}."""
    r = random.Random(seed)
    out = []
    for i in range(n_batches):
        j = i - (n_batches - tt.N_MEAS)
        out.append([(k, v * scale + r.gauss(0, 0.05 if v < 100 else 3.0) + (bump or {}).get((j, idx), 0.0))
                    for idx, (k, v) in enumerate(KERNELS)])
    return out


def _shape(**bumps):
    mixes = ["rud", "main", "hot_next", "deletes", "rud#2"]
    return {m: _timing_proc(n, bump=bumps.get(m.replace("#", "_"))) for n, m in enumerate(mixes)}


def test_timing_clean_shape_passes():
    res = tt.evaluate(_shape(), "rud")
    assert not res["bad"] and res["aside"] is None and not res["rerun"]


def test_timing_stall_batch_is_one_set_aside():
    # one batch of one process: two unrelated kernels over the bound together
    res = tt.evaluate(_shape(hot_next={(4, 0): 24.6, (4, 1): 6.0}), "rud")
    assert not res["bad"], res["bad"]
    assert res["aside"][:2] == ("hot_next", 4) and len(res["aside"][2]) == 2


def test_timing_two_stall_batches_in_one_process_fail_and_rerun():
    res = tt.evaluate(_shape(hot_next={(1, 0): 20.0, (4, 1): 20.0}), "rud")
    assert res["aside"] is None
    assert {(v[1], v[2], v[5]) for v in res["bad"] if v[2] == "batch"} == {("hot_next", "batch", 1),
                                                                           ("hot_next", "batch", 4)}
    assert res["rerun"] == ["hot_next"]
    # the fresh process may not set anything aside
    assert tt.evaluate(_shape(hot_next={(4, 0): 20.0}), "rud", fresh=("hot_next",))["bad"]


def test_timing_excursion_repeated_across_mixes_is_not_set_aside():
    # the same kernel and measured batch in two processes: a draw-tied leak
    res = tt.evaluate(_shape(main={(2, 0): 20.0}, deletes={(2, 0): 20.0}), "rud")
    assert res["aside"] is None and len([v for v in res["bad"] if v[2] == "batch"]) == 2


def test_timing_one_set_aside_per_shape():
    res = tt.evaluate(_shape(main={(2, 0): 20.0}, deletes={(3, 1): 20.0}), "rud")
    assert res["aside"] == ("main", 2, [("k_sort", 20.0)]) or res["aside"][0] == "main"
    assert [v[1] for v in res["bad"] if v[2] == "batch"] == ["deletes"] and res["rerun"] == ["deletes"]


def test_timing_leak_in_every_batch_fails_bias():
    leak = {(j, 0): 3.0 for j in range(tt.N_MEAS)}
    res = tt.evaluate(_shape(deletes=leak), "rud")
    assert any(v[1] == "deletes" and v[2] == "bias" and v[0] == "k_sort" for v in res["bad"]), res["bad"]


def test_timing_slow_reference_process_widens_the_noise():
    # a reference process slow in every batch differs from its second process
    # by as much: that difference is part of the noise, not a failure of
    # every other mix (the r05af case)
    per = _shape()
    per["rud"] = _timing_proc(0, bump={(j, 2): 60.0 for j in range(tt.N_MEAS)})
    res = tt.evaluate(per, "rud")
    assert not res["bad"], res["bad"]


def _interleaved(bump=None, sigma=3.0, offsets=(0.0, 40.0), drift=0.0):
    """Processes of interleaved mixes: {mix: [(block, batch)]}, 3 blocks of 2
    batches per mix; a process offset and a drift per block on the pass."""
    mixes = ["rud", "main", "hot_next", "deletes"]
    procs = []
    for p, off in enumerate(offsets):
        r = random.Random(100 + p)
        per = {m: [] for m in mixes}
        for blk in range(3):
            for m in mixes:
                for j in range(2):
                    per[m].append((blk, [(k, v + (off + drift * blk if v > 100 else 0.0)
                                          + r.gauss(0, sigma if v > 100 else 0.05)
                                          + (bump or {}).get((m, 2 * blk + j, idx), 0.0))
                                         for idx, (k, v) in enumerate(KERNELS)]))
        procs.append(per)
    return procs


def test_interleaved_process_offset_and_drift_cancel():
    lines, bad, mdb = tt.evaluate_interleaved(_interleaved(drift=30.0), "rud")
    assert not bad, bad
    assert mdb["2:k_pass"] < 12.0, mdb  # 40-us process offset, 30-us drift, 3-us batch noise


def test_interleaved_small_leak_in_the_pass_is_seen():
    leak = {("hot_next", j, 2): 12.0 for j in range(6)}
    lines, bad, mdb = tt.evaluate_interleaved(_interleaved(leak, drift=30.0), "rud")
    assert [(v[0], v[1]) for v in bad] == [("k_pass", "hot_next")], bad


def test_interleaved_one_stalled_batch_is_dropped():
    stall = {("main", 3, 0): 25.0}
    lines, bad, mdb = tt.evaluate_interleaved(_interleaved(stall), "rud")
    assert not bad, bad


# ---- the counter test's fresh-process rule (tests/test_oblivious.py)

def test_counter_rerun_candidates():
    mixes = ["main", "rud", "deletes", "hot_next", "main#2"]
    one = [("k_spass", "rud", "batch", 16.4, 3.9, 0, 1), ("k_spass", "rud", "bias", 2.7, 0.6)]
    assert ob.rerun_candidates(one, mixes) == ["rud"]
    assert ob.rerun_candidates(one, mixes, fresh=("rud",)) == []
    # most mixes biased the same way on one kernel: the reference is the suspect
    ref = [("k", m, "bias", -3.0, 1.0) for m in ("rud", "deletes", "hot_next")]
    assert ob.rerun_candidates(ref, mixes) == ["main"]
    # ... and once main has been run again, the violating mixes are
    assert ob.rerun_candidates(ref, mixes, fresh=("main",)) == ["rud", "deletes", "hot_next"]
    # one process failing every launch of a repeated kernel is that process
    rep = [("k_bitonic_tile", "hot_next", "bias", 0.33, 0.25)] * 6 + \
        [("k_copy", "hot_next", "batch", 7.5, 2.56, 3, 4)]
    assert ob.rerun_candidates(rep, mixes) == ["hot_next"]


def test_counter_evaluation_flags_a_one_batch_excursion():
    per = {"main": _proc(_pre([10] * ob.N_MEAS)), "rud": _proc(_pre([10] * ob.N_MEAS)),
           "main#2": _proc(_pre([10] * ob.N_MEAS))}
    per["rud"][3 + 2] = [("k", 1, 1, 100.0 + 16.0, 10.0)]
    lines, bad = ob.evaluate_counters(per)
    assert ("k", "rud", "batch") == bad[0][:3] and bad[0][5] == 2
