"""The gfx950 machine code of one kernel in a built libocn_sw.so, for profile provenance.

A committed counter summary (profiles/sq_valu.json, profiles/pmc_traffic.json) describes one kernel's
dispatches on one workload.  bench.py uses it when it was taken on the same library build
(ocn_build_id) -- or, with ``code_sha`` recorded per kernel, when the loaded library's code for that
kernel is byte for byte the code that was profiled (sha256 of the function's bytes in the gfx950 code
object), so that host-side or other-kernel changes do not void a measurement of unchanged machine code.

Pure Python, no GPU and no ROCm tools: the .hip_fatbin section's clang offload bundle is parsed for
the gfx950 entry, and that ELF's symbol table for the kernel's function bytes.
"""
from __future__ import annotations

import hashlib
import struct

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """{name: (offset, size, addr)} of an ELF64 little-endian image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not an ELF64 little-endian image")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, _typ, _flags, addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        hdrs.append((name, addr, off, size))
    stroff = hdrs[shstrndx][2]
    out = {}
    for i, (name, addr, off, size) in enumerate(hdrs):
        end = elf.index(b"\0", stroff + name)
        out[elf[stroff + name:end].decode()] = (off, size, addr, i)
    return out


def gfx950_code_object(lib_path: str) -> bytes:
    """The gfx950 code object (ELF) bundled in the library's .hip_fatbin section."""
    data = open(lib_path, "rb").read()
    off, size, _addr, _i = _sections(data)[".hip_fatbin"]
    fat = data[off:off + size]
    pos = fat.find(_BUNDLE_MAGIC)
    while pos >= 0:
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith("gfx950"):
                return fat[pos + eoff:pos + eoff + esize]
        pos = fat.find(_BUNDLE_MAGIC, pos + 1)
    raise ValueError("no gfx950 code object in " + lib_path)


def kernel_symbols(code: bytes) -> dict:
    """{mangled name: function bytes} of the code object's function symbols."""
    secs = _sections(code)
    symoff, symsize, _a, _i = secs[".symtab"]
    stroff = secs[".strtab"][0]
    by_index = {v[3]: v for v in secs.values()}
    out = {}
    for k in range(symsize // 24):
        st_name, st_info, _other, shndx, value, size = struct.unpack_from("<IBBHQQ", code, symoff + 24 * k)
        if (st_info & 0xF) != 2 or size == 0 or shndx not in by_index:   # STT_FUNC with bytes
            continue
        end = code.index(b"\0", stroff + st_name)
        name = code[stroff + st_name:end].decode()
        off, _s, addr, _i = by_index[shndx]
        start = off + (value - addr)
        out[name] = code[start:start + size]
    return out


def march_step_symbol(args: str, batched: bool = False) -> str:
    """The mangled name of k_march<MarchStep<args>> (k_march_b with batched), args as in the profile
    summaries: 'true, false, true, false, false, true, false'."""
    bits = "".join("Lb1E" if a.strip() == "true" else "Lb0E" for a in args.split(","))
    if batched:
        return f"_ZN3ocn9k_march_bINS_9MarchStepII{bits}EEEEvNS_10MarchGridBENS_4PackIT_EE".replace("II", "I")
    return f"_ZN3ocn7k_marchINS_9MarchStepII{bits}EEEEvNS_9MarchGridET_".replace("II", "I")


def kernel_code_sha(lib_path: str, symbol: str) -> str | None:
    """sha256 (16 hex digits) of the kernel's machine code in the library, or None if absent."""
    syms = kernel_symbols(gfx950_code_object(lib_path))
    code = syms.get(symbol)
    return hashlib.sha256(code).hexdigest()[:16] if code is not None else None


def sha_by_demangled(lib_path: str, names) -> dict:
    """{demangled kernel name (as rocprofv3 reports it): (mangled symbol, code sha)} for the names found
    in the library (c++filt demangles the code object's symbols; whitespace-insensitive match)."""
    import subprocess
    syms = kernel_symbols(gfx950_code_object(lib_path))
    mangled = sorted(syms)
    dem = subprocess.run(["c++filt"], input="\n".join(mangled), capture_output=True, text=True, check=True).stdout.split("\n")
    key = {"".join(d.split()): m for m, d in zip(mangled, dem)}
    out = {}
    for n in names:
        m = key.get("".join(n.split()))
        if m:
            out[n] = (m, hashlib.sha256(syms[m]).hexdigest()[:16])
    return out

