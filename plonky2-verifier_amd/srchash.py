"""The source hash libp2v.so is built from (tie the binary to the sources).

sha256 over the sorted top-level files of csrc/ (the HIP kernels, the C-ABI and the circuit
compiler: everything libp2v.so is built from) and include/p2v.h, each as
"<relative path>\\0<bytes>\\0"; the first 16 hex digits.  The Makefile compiles the digest into
p2v_version() (csrc/version.cpp); p2v.check_build() recomputes it from the tree the process
runs from and refuses a library built from other sources.  Standard library only: `make` runs
this file as a script.
"""
import hashlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))


def source_files(pkg_dir: str = _HERE):
    csrc = os.path.join(pkg_dir, "csrc")
    files = sorted(os.path.join("csrc", f) for f in os.listdir(csrc) if os.path.isfile(os.path.join(csrc, f)))
    return files + [os.path.join("..", "include", "p2v.h")]


def source_hash(pkg_dir: str = _HERE) -> str:
    h = hashlib.sha256()
    for rel in source_files(pkg_dir):
        with open(os.path.join(pkg_dir, rel), "rb") as f:
            data = f.read()
        h.update(rel.replace(os.sep, "/").encode() + b"\0" + data + b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_hash(sys.argv[1] if len(sys.argv) > 1 else _HERE) + "\n")
