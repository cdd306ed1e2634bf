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
