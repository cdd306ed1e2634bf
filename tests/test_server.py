"""The gRPC front-end and batching server (grapevine_amd/server.py; SURVEY.md
§8(f) rank 4) on CPU: the challenge RNG against openssl's ChaCha20, URI rules
(uri/src/lib.rs:14-26), and the GrapevineAPI Auth/Query flow
(api/proto/grapevine.proto:10-15) end to end over gRPC on 127.0.0.1, with
the store replaced by a test double built from the oracle (the GPU form of
this test, tests/test_gpu_server.py, serves from the HIP store)."""
import json
import os
import random
import threading

import numpy as np
import pytest

from grapevine_amd import abi, wire
from grapevine_amd import server as gs
from grapevine_amd.store import GvsError
from oracle import ffi
from oracle import sr25519 as sr

grpc = pytest.importorskip("grpc")
HERE = os.path.dirname(os.path.abspath(__file__))


def test_challenge_rng_is_chacha20():
    with open(os.path.join(HERE, "golden", "chacha20_openssl.json")) as f:
        vecs = json.load(f)
    for v in vecs:
        r = gs.ChallengeRng(bytes.fromhex(v["key"]))
        ks = b"".join(r.draw(32) for _ in range(10))
        assert ks.hex() == v["keystream"]


def test_uri_rules():
    assert gs.parse_uri("insecure-grapevine://localhost") == ("localhost", 3229, False)
    assert gs.parse_uri("grapevine://example.com/") == ("example.com", 443, True)
    assert gs.parse_uri("insecure-grapevine://10.0.0.1:5555") == ("10.0.0.1", 5555, False)
    assert gs.parse_uri("insecure-grapevine://[::1]:7000") == ("::1", 7000, False)
    for bad in ("http://x", "grapevine:/x", "insecure-grapevine://"):
        with pytest.raises(ValueError):
            gs.parse_uri(bad)


class Signer:
    def __init__(self, rng):
        self.x = rng.randrange(1, sr.L)
        self.public_key = sr.public_key(self.x)
        self.rng = rng

    def sign(self, challenge):
        return sr.sign(self.x, challenge, self.rng.randrange(1, sr.L))


class OracleWireStore:
    """Test double with ObliviousStore.process_wire_batch's contract, built
    from the host codec, oracle/sr25519.py and the seqmodel."""

    def __init__(self, cfg):
        self.model = ffi.Model(cfg)
        self.lock = threading.Lock()

    def process_wire_batch(self, msgs, times, in_stride=None, out_stride=1042, challenges=None):
        q, sig, st = wire.decode_requests(msgs, timestamps=times, strict=False)
        if challenges is not None:
            for k in range(len(msgs)):
                if st[k] == 0 and not sr.verify(bytes(q[k]["auth_identity"]), bytes(challenges[k]),
                                                bytes(sig[k])):
                    q[k]["request_type"] = 0
                    st[k] = abi.WIRE_BAD_SIGNATURE
        with self.lock:
            out = self.model.process_batch(q)
        return [wire.encode_response(r) for r in out], sig, st


def run_clients(store, n_clients=4, rounds=3, window_ms=20.0, on_batch=None):
    """n clients: each creates a message for the next client, then reads its
    own next message, over `rounds` rounds; plus a forged signature, an unknown
    channel and a malformed message.  -> (server, per-client results)."""
    srv = gs.GrapevineServer(store, window_ms=window_ms, clock=lambda: 1_700_000_123,
                             on_batch=on_batch).start()
    uri = f"insecure-grapevine://127.0.0.1:{srv.port}"
    rng = random.Random(3)
    signers = [Signer(random.Random(100 + i)) for i in range(n_clients)]
    clients = [gs.GrapevineClient(uri, s).auth() for s in signers]
    results = [[] for _ in range(n_clients)]
    barrier = threading.Barrier(n_clients)

    def work(i):
        c = clients[i]
        peer = signers[(i + 1) % n_clients].public_key
        for r in range(rounds):
            payload = bytes([i, r]) + rng.randbytes(934)
            resp = c.query(abi.REQUEST_TYPE_CREATE, recipient=peer, payload=payload)
            results[i].append(("create", resp, payload))
            barrier.wait()
            resp = c.query(abi.REQUEST_TYPE_READ)
            results[i].append(("read_next", resp, None))
            barrier.wait()

    th = [threading.Thread(target=work, args=(i,)) for i in range(n_clients)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    # a forged signature: UNAUTHENTICATED; the channel's challenge stream stays in step
    c = clients[0]
    good = bytearray(c.query_bytes(abi.REQUEST_TYPE_READ))
    good[41] ^= 1  # auth_signature byte
    with pytest.raises(grpc.RpcError) as e:
        c.call(bytes(good))
    assert e.value.code() == grpc.StatusCode.UNAUTHENTICATED
    assert c.query(abi.REQUEST_TYPE_READ)["status_code"] in (abi.STATUS_CODE_SUCCESS,
                                                             abi.STATUS_CODE_NOT_FOUND)
    # malformed request bytes: INVALID_ARGUMENT
    c.rng.draw(32)
    with pytest.raises(grpc.RpcError) as e:
        c.call(b"\x0d\x01")
    assert e.value.code() == grpc.StatusCode.INVALID_ARGUMENT
    # unknown channel
    stranger = gs.GrapevineClient(uri, signers[1])
    stranger.cid, stranger.rng = b"\x00" * 16, gs.ChallengeRng(bytes(32))
    with pytest.raises(grpc.RpcError) as e:
        stranger.query(abi.REQUEST_TYPE_READ)
    assert e.value.code() == grpc.StatusCode.UNAUTHENTICATED
    for cl in clients + [stranger]:
        cl.close()
    srv.stop()
    return srv, signers, results


def check_results(signers, results):
    n = len(signers)
    for i, res in enumerate(results):
        for kind, resp, payload in res:
            assert resp["status_code"] == abi.STATUS_CODE_SUCCESS, (i, kind, resp["status_code"])
            if kind == "create":
                assert bytes(resp["record"]["sender"]) == signers[i].public_key
                assert bytes(resp["record"]["payload"]) == payload
                assert resp["record"]["timestamp"] == 1_700_000_123
            else:  # the message the previous client sent me
                assert bytes(resp["record"]["recipient"]) == signers[i].public_key
                assert bytes(resp["record"]["sender"]) == signers[(i - 1) % n].public_key


def test_grpc_flow_over_oracle_double():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024)
    srv, signers, results = run_clients(OracleWireStore(cfg))
    check_results(signers, results)
    assert srv.batches < 3 * 2 * 4 + 4  # calls were batched together


class FailingStore:
    """A store whose batches fail as a whole with a given error code."""

    def __init__(self, code):
        self.code = code

    def process_wire_batch(self, msgs, times, in_stride=None, out_stride=1042, challenges=None):
        raise GvsError(self.code, "injected")


def _one_call(store, on_batch=None):
    srv = gs.GrapevineServer(store, window_ms=1.0, verify=False, on_batch=on_batch,
                             call_timeout=30).start()
    c = gs.GrapevineClient(f"insecure-grapevine://127.0.0.1:{srv.port}", Signer(random.Random(1))).auth()
    with pytest.raises(grpc.RpcError) as e:
        c.query(abi.REQUEST_TYPE_READ)
    c.close()
    return srv, e.value.code()


def test_overflow_is_resource_exhausted_and_server_keeps_serving():
    srv, code = _one_call(FailingStore(abi.GVS_ERR_BATCH_OVERFLOW))
    assert code == grpc.StatusCode.RESOURCE_EXHAUSTED
    assert srv.fatal is None
    srv.stop()


def test_integrity_failure_stops_the_server():
    srv, code = _one_call(FailingStore(abi.GVS_ERR_INTEGRITY))
    assert code == grpc.StatusCode.UNAVAILABLE
    assert srv.fatal and "injected" in srv.fatal
    srv.stop()


def test_on_batch_exception_does_not_kill_the_batcher():
    cfg = abi.make_config(4096, mailbox_partitions=16, mailbox_partition_slots=32, max_batch=1024)

    def boom(*_):
        raise RuntimeError("on_batch failed")

    srv = gs.GrapevineServer(OracleWireStore(cfg), window_ms=1.0, on_batch=boom, call_timeout=30).start()
    c = gs.GrapevineClient(f"insecure-grapevine://127.0.0.1:{srv.port}", Signer(random.Random(1))).auth()
    for _ in range(2):  # the second call is served by the same batcher thread
        assert c.query(abi.REQUEST_TYPE_READ)["status_code"] == abi.STATUS_CODE_NOT_FOUND
    c.close()
    assert len(srv.hook_errors) == 2 and srv.batcher.is_alive()
    srv.stop()
