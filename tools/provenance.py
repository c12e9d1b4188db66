"""Provenance of a measurement or sweep record: which code produced it.

The GPU box receives the tree without .git, so the build writes the commit it was built from
into nanopore-barcoding-orc_amd/dmx/BUILD_INFO.json (Makefile, git-ignored, travels with the
.so files); the record adds the SHA-256 of the libraries actually loaded and of the kernel /
host sources next to them, which identify the code exactly whatever the commit says."""
from __future__ import annotations

import glob
import hashlib
import json
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "nanopore-barcoding-orc_amd")


def _sha(path: str) -> str | None:
    try:
        h = hashlib.sha256()
        with open(path, "rb") as fh:
            for b in iter(lambda: fh.read(1 << 20), b""):
                h.update(b)
        return h.hexdigest()
    except OSError:
        return None


def provenance() -> dict:
    libdmx = os.environ.get("DMX_LIBDMX") or os.path.join(PKG, "dmx", "libdmx.so")
    libdir = os.environ.get("DMX_LIBDIR") or os.path.join(PKG, "dmx")
    out = {"libdmx": os.path.relpath(libdmx, ROOT), "libdmx_sha256": _sha(libdmx),
           "libdmx_io_sha256": _sha(os.path.join(libdir, "libdmx_io.so"))}
    src = hashlib.sha256()
    for p in sorted(glob.glob(os.path.join(PKG, "csrc", "*")) + [os.path.join(ROOT, "include",
                                                                              "dmx.h")]):
        src.update(os.path.basename(p).encode())
        src.update(open(p, "rb").read())
    out["sources_sha256"] = src.hexdigest()
    try:
        with open(os.path.join(PKG, "dmx", "BUILD_INFO.json")) as fh:
            out["build"] = json.load(fh)
    except (OSError, ValueError):
        out["build"] = None
    try:
        out["git_head"] = subprocess.run(["git", "-C", ROOT, "rev-parse", "HEAD"], check=True,
                                         capture_output=True, text=True).stdout.strip()
    except (OSError, subprocess.CalledProcessError):
        out["git_head"] = None   # the GPU box's copy has no .git: see build.git_head
    return out


if __name__ == "__main__":
    print(json.dumps(provenance(), indent=1))
