"""Generate tests/golden/chacha20_openssl.json: ChaCha20 keystream from the
openssl CLI (key, 16-byte IV = 32-bit block counter || 96-bit nonce, all zero
here, so it equals rand_chacha's 64-bit counter / 64-bit stream layout from
block 0).  tests/test_server.py checks grapevine_amd/server.py's
ChallengeRng against it.

    python tests/golden/make_chacha20.py
"""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def main():
    out = []
    with tempfile.TemporaryDirectory() as d:
        for key in (bytes(range(32)), os.urandom(32), os.urandom(32)):
            zin, zout = os.path.join(d, "z"), os.path.join(d, "k")
            with open(zin, "wb") as f:
                f.write(bytes(320))
            subprocess.run(["openssl", "enc", "-chacha20", "-K", key.hex(), "-iv", "00" * 16,
                            "-in", zin, "-out", zout], check=True)
            with open(zout, "rb") as f:
                out.append(dict(key=key.hex(), keystream=f.read().hex()))
    with open(os.path.join(HERE, "chacha20_openssl.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
