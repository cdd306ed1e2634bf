"""gRPC front-end and batching server.

The reference exposes `service GrapevineAPI { rpc Auth(attest.AuthMessage)
returns (AuthMessageWithChallengeSeed); rpc Query(attest.Message) returns
(attest.Message); }` (api/proto/grapevine.proto:10-15) on the URI schemes
grapevine:// (443) and insecure-grapevine:// (3229) (uri/src/lib.rs:14-26).
This module serves that interface and turns the stream of Query calls into
GPU batches: every call waiting when a batching window closes goes through
`gvs_process_wire_batch` (decode, challenge check, the store, encode -- all on
the device), and each caller gets its own response back.

Out of scope: attestation and the Noise channel.  The server
speaks the insecure scheme only: `attest.Message.data` carries the QueryRequest
/ QueryResponse bytes in the clear, and `Auth` returns the 32-byte challenge
seed unencrypted together with a channel id [D].  The challenge RNG is what
README.md:191-199 describes: ChaCha20 seeded with that seed, 32 bytes drawn per
request, in order, on both sides (rand_chacha's ChaCha20Rng: 64-bit block
counter from 0, stream 0; pinned against the openssl CLI's ChaCha20 in
tests/test_server.py).  The attest messages follow mobilecoin's attest.proto
(absent from the reference; `AuthMessage {bytes data = 1}`, `Message {bytes
aad = 1; bytes channel_id = 2; bytes data = 3}` [U]).

Errors: a request the store answers as a hard error (decode failure, wrong
field sizes, a proto fail-fast rule) fails with INVALID_ARGUMENT; a bad
challenge signature with UNAUTHENTICATED; an unknown channel with
UNAUTHENTICATED.  A batch that overflows a fixed bound (nothing applied)
fails its callers with RESOURCE_EXHAUSTED; any other store failure (integrity,
device, exhausted epochs: the handle is dead) fails them with UNAVAILABLE and
stops the server (`fatal` holds the reason).
"""
import concurrent.futures
import os
import queue
import struct
import threading
import time

import numpy as np

from . import abi, wire
from .store import GvsError

SERVICE = "grapevine.GrapevineAPI"
# internal per-call statuses of a batch that failed as a whole
_ST_OVERFLOW, _ST_FATAL = 0xFFFF0001, 0xFFFF0002
SCHEME_SECURE, SCHEME_INSECURE = "grapevine", "insecure-grapevine"
DEFAULT_SECURE_PORT, DEFAULT_INSECURE_PORT = 443, 3229


# ------------------------------------------------------------------ ChaCha20

def _rotl(v, r):
    return ((v << r) | (v >> (32 - r))) & 0xFFFFFFFF


def chacha20_block(key, counter, stream=0):
    """One 64-byte ChaCha20 block: constants, 8 key words, a 64-bit block
    counter and a 64-bit stream id (rand_chacha's layout)."""
    s = [0x61707865, 0x3320646E, 0x79622D32, 0x6B206574, *struct.unpack("<8I", key),
         counter & 0xFFFFFFFF, counter >> 32, stream & 0xFFFFFFFF, stream >> 32]
    x = list(s)

    def qr(a, b, c, d):
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF
        x[d] = _rotl(x[d] ^ x[a], 16)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF
        x[b] = _rotl(x[b] ^ x[c], 12)
        x[a] = (x[a] + x[b]) & 0xFFFFFFFF
        x[d] = _rotl(x[d] ^ x[a], 8)
        x[c] = (x[c] + x[d]) & 0xFFFFFFFF
        x[b] = _rotl(x[b] ^ x[c], 7)

    for _ in range(10):
        qr(0, 4, 8, 12), qr(1, 5, 9, 13), qr(2, 6, 10, 14), qr(3, 7, 11, 15)
        qr(0, 5, 10, 15), qr(1, 6, 11, 12), qr(2, 7, 8, 13), qr(3, 4, 9, 14)
    return struct.pack("<16I", *((x[i] + s[i]) & 0xFFFFFFFF for i in range(16)))


class ChallengeRng:
    """ChaCha20Rng(seed): the per-connection challenge stream (README.md:191-199)."""

    def __init__(self, seed):
        if len(seed) != 32:
            raise ValueError("challenge seed must be 32 bytes")
        self.key, self.counter, self.buf = bytes(seed), 0, b""

    def draw(self, n=32):
        while len(self.buf) < n:
            self.buf += chacha20_block(self.key, self.counter)
            self.counter += 1
        out, self.buf = self.buf[:n], self.buf[n:]
        return out


# --------------------------------------------------------- attest messages [U]

def _ld(field, data):
    n, v = len(data), bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        v.append(b | (0x80 if n else 0))
        if not n:
            break
    return bytes([field << 3 | 2]) + bytes(v) + bytes(data)


def _parse(b, spec, nested=None):
    out = {}
    wire._walk(bytes(b), 0, len(b), spec, out, nested)
    return out


def encode_message(channel_id, data, aad=b""):
    return _ld(1, aad) + _ld(2, channel_id) + _ld(3, data)


def decode_message(b):
    f = _parse(b, {1: 2, 2: 2, 3: 2})
    return f.get(1, b""), f.get(2, b""), f.get(3, b"")


def encode_auth_reply(channel_id, seed):
    return _ld(1, _ld(1, channel_id)) + _ld(2, seed)


def decode_auth_reply(b):
    am = {}
    f = _parse(b, {1: 2, 2: 2}, {1: ({1: 2}, am)})
    return am.get(1, b""), f.get(2, b"")


# ----------------------------------------------------------------------- URIs

def parse_uri(uri):
    """-> (host, port, secure) for grapevine:// / insecure-grapevine:// URIs."""
    scheme, sep, rest = uri.partition("://")
    if not sep or scheme not in (SCHEME_SECURE, SCHEME_INSECURE):
        raise ValueError(f"not a grapevine URI: {uri!r}")
    hostport = rest.split("/", 1)[0]
    secure = scheme == SCHEME_SECURE
    if hostport.startswith("["):
        host, _, tail = hostport[1:].partition("]")
        port = int(tail[1:]) if tail.startswith(":") else None
    elif hostport.count(":") == 1:
        host, p = hostport.split(":")
        port = int(p)
    else:
        host, port = hostport, None
    if not host:
        raise ValueError(f"no host in {uri!r}")
    return host, port or (DEFAULT_SECURE_PORT if secure else DEFAULT_INSECURE_PORT), secure


# --------------------------------------------------------------------- server

class _Pending:
    __slots__ = ("data", "challenge", "done", "response", "status")

    def __init__(self, data, challenge):
        self.data, self.challenge = data, challenge
        self.done = threading.Event()
        self.response, self.status = None, None


class GrapevineServer:
    """GrapevineAPI over a store with `process_wire_batch` (an ObliviousStore).

    window_ms: how long the batcher waits after the first request of a batch
    for more; max_batch: the most requests per GPU batch.  on_batch(msgs,
    times, challenges, responses, statuses), if given, sees every batch (tests
    replay them into the oracle)."""

    def __init__(self, store, address="127.0.0.1:0", window_ms=2.0, max_batch=1024,
                 verify=True, clock=None, on_batch=None, workers=64, call_timeout=60.0):
        import grpc
        self.grpc = grpc
        self.store, self.window, self.max_batch = store, window_ms * 1e-3, max_batch
        self.verify, self.on_batch = verify, on_batch
        self.clock = clock or (lambda: int(time.time()))
        self.channels, self.lock = {}, threading.Lock()
        self.q = queue.Queue()
        self.stop_evt = threading.Event()
        self.batches = 0
        self.fatal = None  # set when the store failed for good
        self.hook_errors = []  # exceptions raised by on_batch
        self.call_timeout = call_timeout
        self.server = grpc.server(concurrent.futures.ThreadPoolExecutor(max_workers=workers))
        handler = grpc.method_handlers_generic_handler(SERVICE, {
            "Auth": grpc.unary_unary_rpc_method_handler(self._auth),
            "Query": grpc.unary_unary_rpc_method_handler(self._query),
        })
        self.server.add_generic_rpc_handlers((handler,))
        self.port = self.server.add_insecure_port(address)
        self.batcher = threading.Thread(target=self._run, name="gvs-batcher", daemon=True)

    def start(self):
        self.batcher.start()
        self.server.start()
        return self

    def stop(self):
        self.server.stop(grace=None)
        self.stop_evt.set()
        self.q.put(None)
        self.batcher.join()

    # -- rpc handlers (gRPC worker threads) --
    def _auth(self, request, context):
        seed, cid = os.urandom(32), os.urandom(16)
        with self.lock:
            self.channels[cid] = (ChallengeRng(seed), threading.Lock())
        return encode_auth_reply(cid, seed)

    def _query(self, request, context):
        grpc = self.grpc
        try:
            _, cid, data = decode_message(request)
        except ValueError:
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "malformed attest.Message")
        with self.lock:
            ch = self.channels.get(cid)
        if ch is None:
            context.abort(grpc.StatusCode.UNAUTHENTICATED, "unknown channel: call Auth first")
        rng, ch_lock = ch
        if len(data) > abi.WIRE_SLOT_MAX:
            with ch_lock:
                rng.draw(32)  # the client drew one for this request too
            context.abort(grpc.StatusCode.INVALID_ARGUMENT, "request larger than a wire slot")
        if self.fatal is not None:
            context.abort(grpc.StatusCode.UNAVAILABLE, f"store failed: {self.fatal}")
        with ch_lock:  # draw and enqueue together: the channel's requests keep their order
            p = _Pending(data, rng.draw(32))
            self.q.put(p)
        if not p.done.wait(self.call_timeout):
            context.abort(grpc.StatusCode.DEADLINE_EXCEEDED, "batcher did not answer")
        if p.response:
            return encode_message(cid, p.response)
        if p.status == abi.WIRE_BAD_SIGNATURE:
            context.abort(grpc.StatusCode.UNAUTHENTICATED, "challenge signature does not verify")
        if p.status == _ST_OVERFLOW:
            context.abort(grpc.StatusCode.RESOURCE_EXHAUSTED, "batch overflowed a fixed bound; retry")
        if p.status == _ST_FATAL:
            context.abort(grpc.StatusCode.UNAVAILABLE, f"store failed: {self.fatal}")
        context.abort(grpc.StatusCode.INVALID_ARGUMENT, "request rejected (grapevine.proto:57-64)")

    # -- batcher --
    def _run(self):
        while not self.stop_evt.is_set():
            first = self.q.get()
            if first is None:
                break
            batch = [first]
            deadline = time.monotonic() + self.window
            while len(batch) < self.max_batch:
                left = deadline - time.monotonic()
                if left <= 0:
                    break
                try:
                    p = self.q.get(timeout=left)
                except queue.Empty:
                    break
                if p is None:
                    self.stop_evt.set()
                    break
                batch.append(p)
            self._serve(batch)

    def _serve(self, batch):
        msgs = [p.data for p in batch]
        now = self.clock()
        times = np.full(len(batch), now, np.uint64)
        chal = np.frombuffer(b"".join(p.challenge for p in batch), np.uint8).reshape(-1, 32)
        resp, status = [b""] * len(batch), np.full(len(batch), _ST_FATAL, np.uint32)
        try:
            try:
                resp, _, status = self.store.process_wire_batch(
                    msgs, times, challenges=chal if self.verify else None)
            except GvsError as e:
                if e.code == abi.GVS_ERR_BATCH_OVERFLOW:
                    # nothing was applied: the callers may retry
                    status = np.full(len(batch), _ST_OVERFLOW, np.uint32)
                else:
                    # integrity failure, device error, exhausted epochs: the
                    # handle refuses every further call, so stop serving
                    self._fail(e)
            except Exception as e:  # noqa: BLE001 - anything else is a server fault
                self._fail(e)
            self.batches += 1
            if self.on_batch:
                try:
                    self.on_batch(msgs, times, chal, resp, status)
                except Exception as e:  # noqa: BLE001 - a hook must not kill the batcher
                    self.hook_errors.append(e)
        finally:  # every caller is answered, whatever on_batch or the store did
            for p, r, s in zip(batch, resp, status):
                p.response, p.status = r, int(s)
                p.done.set()

    def _fail(self, err):
        """A store error that poisons the handle: refuse new calls and stop the
        gRPC server (its process should exit non-zero; `fatal` says why)."""
        self.fatal = f"{type(err).__name__}: {err}"
        self.stop_evt.set()
        threading.Thread(target=self.server.stop, args=(None,), daemon=True).start()


# --------------------------------------------------------------------- client

class GrapevineClient:
    """A client of the insecure scheme: Auth, then Query calls signed over the
    channel's challenge stream.  `signer` has `.public_key` (32 B) and
    `.sign(challenge) -> 64 B` (mc-crypto-keys' sign_schnorrkel under the
    context "grapevine-challenge")."""

    def __init__(self, uri, signer):
        import grpc
        host, port, secure = parse_uri(uri)
        if secure:
            raise NotImplementedError("grapevine:// needs the attested Noise channel (out of scope)")
        self.ch = grpc.insecure_channel(f"{host}:{port}")
        self._auth = self.ch.unary_unary(f"/{SERVICE}/Auth")
        self._query = self.ch.unary_unary(f"/{SERVICE}/Query")
        self.signer = signer
        self.cid, self.rng = None, None

    def auth(self):
        cid, seed = decode_auth_reply(self._auth(_ld(1, b"")))
        self.cid, self.rng = cid, ChallengeRng(seed)
        return self

    def query_bytes(self, request_type, msg_id=bytes(16), recipient=bytes(32), payload=bytes(936)):
        """A canonical QueryRequest for this client's identity, signed over the
        next challenge."""
        sig = self.signer.sign(self.rng.draw(32))
        q = np.zeros(1, abi.REQUEST_DTYPE)
        q["request_type"] = request_type
        q["auth_identity"] = np.frombuffer(self.signer.public_key, np.uint8)
        q["msg_id"] = np.frombuffer(bytes(msg_id), np.uint8)
        q["recipient"] = np.frombuffer(bytes(recipient), np.uint8)
        q["payload"] = np.frombuffer(bytes(payload), np.uint8)
        return wire.encode_requests(q, np.frombuffer(sig, np.uint8).reshape(1, 64))[0].tobytes()

    def call(self, request_bytes, timeout=60):
        """Send raw QueryRequest bytes -> QueryResponse bytes (raises grpc.RpcError)."""
        _, _, data = decode_message(self._query(encode_message(self.cid, request_bytes), timeout=timeout))
        return data

    def query(self, request_type, **fields):
        """-> gvs_response (numpy record) of the decoded QueryResponse."""
        return wire.decode_responses([self.call(self.query_bytes(request_type, **fields))])[0]

    def close(self):
        self.ch.close()
