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
* write the new bundle at the old one's offset and zero the rest of its
  length. The ELF layout is untouched (no section or segment moves), each
  registration wrapper still points at a bundle, and the zero tail costs
  nothing in a compressed image layer.

A library built without -fgpu-rdc holds one bundle per source file, back to
back in the section: each is cut at its own offset (``bundles``).

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


MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def bundle_bytes(data: bytes) -> int:
    """Length of the offload bundle at the start of ``data``: a compressed
    bundle (``CCOB``) records its total size (v2: u32, v3: u64 at byte 8),
    which excludes the zero tail an earlier strip left; an uncompressed one
    ends with its last entry (the entry table: u64 count, then per entry u64
    offset, u64 size, u64 triple length, triple); anything else: all of it."""
    if data[:4] == b"CCOB":
        version, = struct.unpack_from("<H", data, 4)
        if version == 2:
            return struct.unpack_from("<I", data, 8)[0]
        if version >= 3:
            return struct.unpack_from("<Q", data, 8)[0]
    if data[:len(MAGIC)] == MAGIC and len(data) >= len(MAGIC) + 8:
        count, = struct.unpack_from("<Q", data, len(MAGIC))
        pos = end = len(MAGIC) + 8
        for _ in range(count):
            if pos + 24 > len(data):
                return len(data)
            eoff, esize, tlen = struct.unpack_from("<QQQ", data, pos)
            pos += 24 + tlen
            end = max(end, eoff + esize)
        return min(max(end, pos), len(data))
    return len(data)


def bundles(data: bytes) -> list[tuple[int, int]]:
    """(offset, length) of every offload bundle in a ``.hip_fatbin`` section.
    A library built with -fgpu-rdc (librccl) holds one; one built without it
    holds one per source file, back to back at aligned offsets, each registered
    by its own __hipRegisterFatBinary wrapper at that offset. The
    gaps between them (alignment padding, an earlier strip's zero tail) must be
    zero; anything else raises, rather than guess at a layout."""
    out, i = [], 0
    while i < len(data):
        starts = [j for j in (data.find(b"CCOB", i), data.find(MAGIC, i)) if j >= 0]
        if not starts:
            if any(data[i:]):
                raise ValueError(f"non-zero bytes after the last bundle at offset {i}")
            break
        j = min(starts)
        if any(data[i:j]):
            raise ValueError(f"non-zero bytes between bundles at offsets {i}..{j}")
        n = bundle_bytes(data[j:])
        if n <= 0:
            raise ValueError(f"empty bundle at offset {j}")
        out.append((j, n))
        i = j + n
    return out


def targets(bundler: str, bundle: str) -> list[str]:
    out = subprocess.run([bundler, "--list", "--type=o", f"--input={bundle}"],
                         capture_output=True, text=True, check=True).stdout
    return [t.strip() for t in out.splitlines() if t.strip()]


def _strip_one(data: bytes, target: str, bundler: str, td: str, tag: str) -> dict:
    """Re-bundle one offload bundle as host + ``target`` only, compressed.
    Returns {"blob": bytes} or {"reason": why it is kept as is}, plus targets."""
    src = os.path.join(td, f"fatbin{tag}.bin")
    with open(src, "wb") as f:
        f.write(data)
    tg = targets(bundler, src)
    dev = [t for t in tg if t.endswith("--" + target) or t.endswith("--" + target + ":xnack-")]
    res = {"targets": len(tg)}
    if not dev:
        return {**res, "reason": f"no {target} code object in the bundle"}
    keep = [t for t in tg if t == HOST] + dev[:1]
    if len(keep) == len(tg):
        return {**res, "reason": "bundle holds no other target"}
    outs = [os.path.join(td, f"part{tag}_{i}") for i in range(len(keep))]
    subprocess.run([bundler, "--unbundle", "--type=o", f"--input={src}",
                    "--targets=" + ",".join(keep)] + [f"--output={o}" for o in outs],
                   check=True)
    new = os.path.join(td, f"new{tag}.bin")
    subprocess.run([bundler, "--type=o", "--compress", "--targets=" + ",".join(keep),
                    f"--output={new}"] + [f"--input={o}" for o in outs], check=True)
    with open(new, "rb") as f:
        blob = f.read()
    if len(blob) > len(data):
        return {**res, "reason": "re-bundled code is larger than the bundle"}
    return {**res, "blob": blob, "kept": keep, "dropped": len(tg) - len(keep)}


def strip(lib: str, target: str, bundler: str, dry_run: bool = False) -> dict:
    """Cut every offload bundle of ``lib``'s .hip_fatbin to host + ``target``,
    each rewritten at its own offset and zero-filled to its old length (the
    registration wrappers keep pointing at valid bundles)."""
    res = {"lib": os.path.basename(lib), "bytes": os.path.getsize(lib)}
    sec = section(lib)
    if sec is None:
        return {**res, "changed": False, "reason": "no .hip_fatbin section"}
    off, size = sec
    with open(lib, "rb") as f:
        f.seek(off)
        data = f.read(size)
    try:
        found = bundles(data)
    except ValueError as e:
        return {**res, "changed": False, "reason": f"unrecognised section layout: {e}"}
    res.update(section_bytes=size, bundles=len(found))
    if not found:
        return {**res, "changed": False, "reason": "no offload bundle in the section"}
    writes, reasons, kept, dropped, total_tg = [], [], None, 0, 0
    with tempfile.TemporaryDirectory() as td:
        for i, (b0, n) in enumerate(found):
            r = _strip_one(data[b0:b0 + n], target, bundler, td, str(i))
            total_tg = max(total_tg, r["targets"])
            if "blob" in r:
                writes.append((b0, n, r["blob"]))
                kept, dropped = r["kept"], dropped + r["dropped"]
            else:
                reasons.append(r["reason"])
    res["targets"] = total_tg
    if not writes:
        return {**res, "changed": False, "reason": reasons[0]}
    if not dry_run:
        with open(lib, "r+b") as f:
            for b0, n, blob in writes:
                f.seek(off + b0)
                f.write(blob)
                f.write(bytes(n - len(blob)))
    out = {**res, "changed": not dry_run, "kept": kept,
           "bundle_bytes": sum(len(w[2]) for w in writes),
           "rewritten_bundles": len(writes),
           "dropped_targets": dropped // len(writes)}
    if reasons:
        out["unchanged_bundles"] = reasons
    return out


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
