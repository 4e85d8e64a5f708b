"""Identity of the native sources a measurement was taken on: a SHA-256 over the contents of every file the
library is built from (csrc/ and include/, sorted by path). bench.py reports PMC-derived numbers from
profiles/ only when the file carries the hash of the tree being benchmarked."""
from __future__ import annotations

import hashlib
import os

_PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_ROOT = os.path.dirname(_PKG)
_EXT = (".hip", ".cpp", ".h", "Makefile")


def source_tree_hash() -> str:
    h = hashlib.sha256()
    files = []
    for d in (os.path.join(_PKG, "csrc"), os.path.join(_ROOT, "include")):
        for name in sorted(os.listdir(d)):
            if name.endswith(_EXT):
                files.append(os.path.join(d, name))
    for f in files:
        h.update(os.path.relpath(f, _ROOT).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]
