#!/usr/bin/env python3
"""Keep only the gfx950 device code in a shared library's HIP fat binary.

ROCm's librccl.so carries one compressed offload bundle (``CCOB``) in its
``.hip_fatbin`` section with code objects for 13 GPU targets (gfx908 ..
gfx1201): 570 MB of the validation image's 775 MB runtime closure, and at
run time the HIP runtime decompresses that bundle before it can pick out the
gfx950 code object RCCL's first kernel launch needs. The image only ever runs
on MI355X, so ``collect-runtime.sh`` rewrites the section in place:

* unbundle the host entry and the gfx950 code object
  (``clang-offload-bundler --unbundle``),
* re-bundle just those two, compressed (``--compress``),
* write the new bundle at the section's start and zero the rest of the
  section. The ELF layout is untouched (no section or segment moves), the
  runtime's registration still points at the section start, and the zero
  tail costs nothing in a compressed image layer.

Libraries without a ``.hip_fatbin`` section, or whose bundle holds no other
target, are copied unchanged. usage: strip-fatbin.py LIB [--target gfx950]
[--bundler PATH] [--dry-run]  (rewrites LIB in place; prints one JSON line)
"""
from __future__ import annotations

import argparse
import json
import os
import struct
import subprocess
import sys
import tempfile

HOST = "host-x86_64-unknown-linux-gnu-"


def section(path: str, name: str = ".hip_fatbin") -> tuple[int, int] | None:
    """(file offset, size) of an ELF64 little-endian section, None if absent."""
    with open(path, "rb") as f:
        ident = f.read(64)
        if ident[:4] != b"\x7fELF" or ident[4] != 2 or ident[5] != 1:
            raise ValueError(f"{path}: not a little-endian ELF64 file")
        shoff, = struct.unpack_from("<Q", ident, 0x28)
        shentsize, shnum, shstrndx = struct.unpack_from("<HHH", ident, 0x3A)
        f.seek(shoff)
        hdrs = [f.read(shentsize) for _ in range(shnum)]
        _, _, _, _, str_off, str_size = struct.unpack_from("<IIQQQQ", hdrs[shstrndx])
        f.seek(str_off)
        names = f.read(str_size)
        for h in hdrs:
            nm, _typ, _flags, _addr, off, size = struct.unpack_from("<IIQQQQ", h)
            if names[nm:names.index(b"\0", nm)].decode() == name:
                return off, size
    return None


def bundle_bytes(data: bytes) -> int:
    """Length of the offload bundle at the start of ``data``: a compressed
    bundle (``CCOB``) records its total size (v2: u32, v3: u64 at byte 8),
    which excludes the zero tail an earlier strip left; otherwise all of it."""
    if data[:4] == b"CCOB":
        version, = struct.unpack_from("<H", data, 4)
        if version == 2:
            return struct.unpack_from("<I", data, 8)[0]
        if version >= 3:
            return struct.unpack_from("<Q", data, 8)[0]
    return len(data)


def targets(bundler: str, bundle: str) -> list[str]:
    out = subprocess.run([bundler, "--list", "--type=o", f"--input={bundle}"],
                         capture_output=True, text=True, check=True).stdout
    return [t.strip() for t in out.splitlines() if t.strip()]


def strip(lib: str, target: str, bundler: str, dry_run: bool = False) -> dict:
    res = {"lib": os.path.basename(lib), "bytes": os.path.getsize(lib)}
    sec = section(lib)
    if sec is None:
        return {**res, "changed": False, "reason": "no .hip_fatbin section"}
    off, size = sec
    with tempfile.TemporaryDirectory() as td:
        src = os.path.join(td, "fatbin.bin")
        with open(lib, "rb") as f:
            f.seek(off)
            data = f.read(size)
        data = data[:bundle_bytes(data)]
        with open(src, "wb") as f:
            f.write(data)
        tg = targets(bundler, src)
        dev = [t for t in tg if t.endswith("--" + target) or t.endswith("--" + target + ":xnack-")]
        res.update(section_bytes=size, targets=len(tg))
        if not dev:
            return {**res, "changed": False, "reason": f"no {target} code object in the bundle"}
        keep = [t for t in tg if t == HOST] + dev[:1]
        if len(keep) == len(tg):
            return {**res, "changed": False, "reason": "bundle holds no other target"}
        outs = [os.path.join(td, f"part{i}") for i in range(len(keep))]
        subprocess.run([bundler, "--unbundle", "--type=o", f"--input={src}",
                        "--targets=" + ",".join(keep)] + [f"--output={o}" for o in outs],
                       check=True)
        new = os.path.join(td, "new.bin")
        subprocess.run([bundler, "--type=o", "--compress", "--targets=" + ",".join(keep),
                        f"--output={new}"] + [f"--input={o}" for o in outs], check=True)
        with open(new, "rb") as f:
            blob = f.read()
        if len(blob) > size:
            return {**res, "changed": False, "reason": "re-bundled code is larger than the section"}
        if not dry_run:
            with open(lib, "r+b") as f:
                f.seek(off)
                f.write(blob)
                f.write(bytes(size - len(blob)))
        return {**res, "changed": not dry_run, "kept": keep, "bundle_bytes": len(blob),
                "dropped_targets": len(tg) - len(keep)}


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("lib")
    ap.add_argument("--target", default="gfx950")
    ap.add_argument("--bundler", default="/opt/rocm/lib/llvm/bin/clang-offload-bundler")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    print(json.dumps(strip(a.lib, a.target, a.bundler, a.dry_run)))
    return 0


if __name__ == "__main__":
    sys.exit(main())
