"""Generate tests/golden/ed25519_openssl.json: Ed25519 keys, messages and
signatures made by the openssl CLI (an independent implementation of the
edwards25519 group that ristretto255 is built on).  tests/test_sr25519.py
checks oracle/sr25519.py's curve arithmetic against them.

    python tests/golden/make_ed25519.py
"""
import json
import os
import subprocess
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def main(n=8):
    out = []
    with tempfile.TemporaryDirectory() as d:
        for i in range(n):
            key, msg, sig = (os.path.join(d, f) for f in ("k.pem", "m.bin", "s.bin"))
            subprocess.run(["openssl", "genpkey", "-algorithm", "ed25519", "-out", key], check=True)
            der = subprocess.run(["openssl", "pkey", "-in", key, "-pubout", "-outform", "DER"],
                                 check=True, capture_output=True).stdout
            m = os.urandom(17 * i + 3)
            with open(msg, "wb") as f:
                f.write(m)
            subprocess.run(["openssl", "pkeyutl", "-sign", "-inkey", key, "-rawin", "-in", msg,
                            "-out", sig], check=True)
            with open(sig, "rb") as f:
                s = f.read()
            out.append(dict(pk=der[-32:].hex(), msg=m.hex(), sig=s.hex()))
    with open(os.path.join(HERE, "ed25519_openssl.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
