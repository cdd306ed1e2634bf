"""The gRPC front-end serving from the HIP store (grapevine_amd/server.py over
ObliviousStore.process_wire_batch): the Auth/Query flow of tests/test_server.py
end to end, and every GPU batch the server formed replayed through the oracle
double -- responses and statuses bit-exact."""
import numpy as np
import pytest

from grapevine_amd import abi
from grapevine_amd.store import ObliviousStore

from test_server import OracleWireStore, check_results, run_clients

pytestmark = pytest.mark.gpu
pytest.importorskip("grpc")


def test_grpc_flow_on_gpu_store_bit_exact():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024)
    store = ObliviousStore(cfg)
    double = OracleWireStore(cfg)
    mismatches, seen = [], []

    def replay(msgs, times, chal, resp, status):
        want, _, wst = double.process_wire_batch(msgs, times, challenges=chal)
        seen.append(len(msgs))
        if list(resp) != want or not np.array_equal(status, wst):
            mismatches.append((len(seen), [k for k in range(len(msgs)) if resp[k] != want[k]][:5]))

    srv, signers, results = run_clients(store, on_batch=replay)
    check_results(signers, results)
    assert not mismatches, mismatches
    assert sum(seen) == 4 * 3 * 2 + 3 and len(seen) < sum(seen)  # + forged, read, malformed
    st = store.stats()
    assert (st["messages"], st["mailboxes"]) == (double.model.messages, double.model.mailboxes)
    store.close()
