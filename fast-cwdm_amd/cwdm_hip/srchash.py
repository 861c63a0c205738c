"""Hash of the native sources libcwdm.so is built from.

The Makefile bakes ``source_hash()`` into the library (``cwdm_build_id()``);
``smoke()`` and the CPU tests recompute it from the tree and refuse a library
built from other sources (the .so travels to the GPU box untracked, so this is
what ties it to the committed kernels).  Runnable as a script: the Makefile
calls ``python3 srchash.py``.
"""
import hashlib
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.normpath(os.path.join(_HERE, "..", "csrc"))
HEADER = os.path.normpath(os.path.join(_HERE, "..", "..", "include", "cwdm.h"))


def source_files():
    names = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".hpp")) or f == "Makefile")
    return [os.path.join(CSRC, f) for f in names] + [HEADER]


def source_hash():
    h = hashlib.sha256()
    for path in source_files():
        h.update(os.path.basename(path).encode())
        h.update(b"\0")
        with open(path, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


if __name__ == "__main__":
    print(source_hash())
