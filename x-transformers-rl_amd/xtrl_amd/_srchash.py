"""Content hash of the HIP / C++ sources libxtrl_hip.so is built from (csrc/* and include/xtrl_hip.h).

The Makefile compiles it into the library (xtrl_source_hash()); xtrl_amd._lib compares it with the
sources in the tree at load time, so a library built from other sources than the ones beside it
fails loudly instead of running.  Run as a script it prints the hash (used by the Makefile)."""
from __future__ import annotations

import hashlib
from pathlib import Path

PKG = Path(__file__).resolve().parent.parent          # x-transformers-rl_amd/


def source_files():
    files = sorted(p for p in (PKG / 'csrc').iterdir() if p.suffix in ('.hip', '.h', '.cpp'))
    return files + [PKG.parent / 'include' / 'xtrl_hip.h']


def source_hash():
    h = hashlib.sha1()
    for p in source_files():
        h.update(p.name.encode() + b'\0' + p.read_bytes() + b'\0')
    return h.hexdigest()[:16]


if __name__ == '__main__':
    print(source_hash())
