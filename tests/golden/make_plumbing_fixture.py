#!/usr/bin/env python3
"""Capture the plumbing-config fixture: tests/golden/plumbing_echoes.npz.

BASELINE configs[0] is the reference's stress server echoing 1500-byte-MTU data
segments over loopback, every TCP check computed on the CPU by
csum_continue(getPseudoHeaderSum(...)) (/root/reference/context.c:104-145,
called at :208-209) on segments framed as send_packet frames them
(context.c:169-206). tests/c/raw_echo runs that configuration here (it needs
raw sockets: root or a user namespace — the GPU pool has neither, so the
capture is committed): its server frames every echo of a 1456-byte payload
that way and fills the check on the CPU ("cpu" mode); the kernel fills the
IPv4 id and header checksum of each IPPROTO_RAW send; a raw sniffer on lo
records each echo as it crossed the wire.

Stored (numpy .npz, no pickles): `wire` the sniffed echoes back to back, `off`
and `length` per echo, plus the run's JSON summary. Regenerate with
    make tests/c/raw_echo && python3 tests/golden/make_plumbing_fixture.py [n]
"""
import json
import os
import struct
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main(n: int = 256) -> None:
    exe = os.path.join(REPO, "tests", "c", "raw_echo")
    env = {k: v for k, v in os.environ.items() if k != "LD_PRELOAD" and not k.startswith("TCPCSUM_PRELOAD")}
    with tempfile.TemporaryDirectory() as td:
        path = os.path.join(td, "echo.bin")
        r = subprocess.run([exe, str(n), path, "cpu"], env=env, capture_output=True, text=True, timeout=120)
        if r.returncode != 0:
            sys.exit(f"raw_echo failed ({r.returncode}): {r.stdout}{r.stderr}")
        summary = json.loads(r.stdout.strip().splitlines()[-1])
        data = open(path, "rb").read()
    wire, off, length = bytearray(), [], []
    pos = 0
    while pos < len(data):
        (lo,) = struct.unpack_from("<I", data, pos)
        pos += 4 + lo                        # the packet as built (check filled by the server's CPU)
        (li,) = struct.unpack_from("<I", data, pos)
        got = data[pos + 4:pos + 4 + li]     # the packet as sniffed on lo
        pos += 4 + li
        off.append(len(wire))
        length.append(li)
        wire += got
    assert len(off) == n, (len(off), n)
    np.savez_compressed(os.path.join(HERE, "plumbing_echoes.npz"), wire=np.frombuffer(bytes(wire), np.uint8),
                        off=np.array(off, np.uint64), length=np.array(length, np.uint32),
                        summary=np.frombuffer(json.dumps(summary).encode(), np.uint8))
    print(f"wrote {n} echoes ({len(wire)} bytes): {summary}")


if __name__ == "__main__":
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 256)
