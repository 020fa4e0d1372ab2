"""Build identity of libncf_hip.so (no torch import: build_ext.sh runs it before anything else).

Two hashes are compiled into the library (``ncf_build_info()``, include/ncf_hip.h) and checked by
``_lib.load()`` before any entry point is bound:

* ``abi``: the C-ABI table the Python side binds (``_lib.SIGNATURES``: names, result and
  argument types, in order).  A library built from another table would take its arguments in
  the wrong slots; it is refused.
* ``src``: the kernel sources the library was compiled from (``csrc/*.hip``, ``csrc/*.h``,
  ``include/ncf_hip.h``).  A library older or newer than the sources beside it — rebuilt while a
  GPU call waited in the queue, or not rebuilt after an edit — is refused too (when the sources
  are present; an installed package without them skips this half).

    python _abi.py abi      # the hash of _lib.SIGNATURES
    python _abi.py src [DIR]  # the hash of the sources (DIR: another csrc tree, A/B builds)
"""
import ctypes
import hashlib
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
HEADER = os.path.join(HERE, "..", "include", "ncf_hip.h")

_CODE = {ctypes.c_void_p: "p", ctypes.c_int64: "l", ctypes.c_int: "i", ctypes.c_int32: "i",
         ctypes.c_float: "f", ctypes.c_double: "d", ctypes.c_uint64: "u",
         ctypes.c_char_p: "s"}


def load_signatures():
    """SIGNATURES of _lib.py without importing torch (exec of the table only)."""
    src = open(os.path.join(HERE, "_lib.py")).read()
    start = src.index("P = ctypes.c_void_p")
    end = src.index("\nclass ReduceDesc")
    ns = {"ctypes": ctypes}
    exec(src[start:end], ns)
    return ns["SIGNATURES"]


def abi_hash(signatures) -> str:
    text = ";".join(f"{n}:{_CODE[r]}:{''.join(_CODE[a] for a in args)}"
                    for n, (r, args) in signatures.items())
    return hashlib.sha256(text.encode()).hexdigest()[:16]


def source_files(csrc: str = CSRC):
    if not os.path.isdir(csrc):
        return []
    fs = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                if f.endswith((".hip", ".h")))
    if os.path.exists(HEADER):
        fs.append(HEADER)
    return fs


def src_hash(csrc: str = CSRC) -> str:
    """'' when the sources are not present."""
    fs = source_files(csrc)
    if not fs:
        return ""
    h = hashlib.sha256()
    for f in fs:
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    what = sys.argv[1] if len(sys.argv) > 1 else "abi"
    print(abi_hash(load_signatures()) if what == "abi"
          else src_hash(sys.argv[2] if len(sys.argv) > 2 else CSRC))
