"""Per-kernel identity of the gfx950 machine code inside libprt.so.

A committed PMC summary (profiles/*_current.json) prices one build of a kernel.  To tell whether the library
being timed is that build, both sides hash the kernel's own machine code: the clang offload bundles in the
library's `.hip_fatbin` section are split into their gfx950 code objects, and in each code object the
kernel's function bytes (`.text`, from its symbol's value and size) plus its 64-byte kernel descriptor
(`<name>.kd`: register counts, LDS size, scratch) are hashed.  Pure ELF parsing on the host: nothing is
loaded or launched.
"""
import hashlib
import struct

_BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf):
    """{name: (offset, size, addr)} of a 64-bit little-endian ELF image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2 or elf[5] != 1:
        raise ValueError("not a 64-bit little-endian ELF")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = [struct.unpack_from("<IIQQQQIIQQ", elf, shoff + i * shentsize) for i in range(shnum)]
    stroff = hdrs[shstrndx][4]
    out = {}
    for h in hdrs:
        name_end = elf.index(b"\0", stroff + h[0])
        out[elf[stroff + h[0]:name_end].decode()] = (h[4], h[5], h[3])
    return out


def _symbols(elf, secs):
    """[(name, value, size)] from .symtab."""
    off, size, _ = secs[".symtab"]
    stroff = secs[".strtab"][0]
    syms = []
    for i in range(size // 24):
        st_name, _info, _other, _shndx, value, sz = struct.unpack_from("<IBBHQQ", elf, off + 24 * i)
        end = elf.index(b"\0", stroff + st_name)
        syms.append((elf[stroff + st_name:end].decode(), value, sz))
    return syms


def _code_objects(lib_bytes, arch):
    """Every `arch` code object in the offload bundles of the `.hip_fatbin` section."""
    secs = _sections(lib_bytes)
    if ".hip_fatbin" not in secs:
        raise ValueError("no .hip_fatbin section")
    off, size, _ = secs[".hip_fatbin"]
    fat = lib_bytes[off:off + size]
    pos, objs = 0, []
    while True:
        pos = fat.find(_BUNDLE_MAGIC, pos)
        if pos < 0:
            return objs
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if triple.endswith(arch) and esize:
                objs.append(fat[pos + eoff:pos + eoff + esize])
        pos = p


def _vaddr_to_off(secs, addr):
    for off, size, base in secs.values():
        if base and base <= addr < base + size:
            return off + addr - base
    raise ValueError(f"address {addr:#x} in no section")


def kernel_hashes(lib_path, arch="gfx950"):
    """{mangled kernel name: sha256 hex of its machine code + kernel descriptor} for every kernel in the
    library's `arch` code objects."""
    with open(lib_path, "rb") as f:
        lib = f.read()
    out = {}
    for co in _code_objects(lib, arch):
        secs = _sections(co)
        syms = {name: (val, sz) for name, val, sz in _symbols(co, secs)}
        for name, (val, sz) in syms.items():
            if not name.endswith(".kd") or name[:-3] not in syms:
                continue
            fval, fsz = syms[name[:-3]]
            h = hashlib.sha256()
            fo = _vaddr_to_off(secs, fval)
            h.update(co[fo:fo + fsz])
            ko = _vaddr_to_off(secs, val)
            h.update(co[ko:ko + sz])
            out[name[:-3]] = h.hexdigest()
    return out


def demangled_base(name):
    """`_ZN3prt8k_trace2ILi32E...` -> `k_trace2` (the bare kernel name, enough to pick a kernel)."""
    if not name.startswith("_ZN"):
        return name
    p, parts = 3, []
    while p < len(name) and name[p].isdigit():
        q = p
        while name[q].isdigit():
            q += 1
        n = int(name[p:q])
        parts.append(name[q:q + n])
        p = q + n
    return parts[-1] if parts else name


def kernel_hash(lib_path, kernel, arch="gfx950"):
    """{mangled name: hash} of every instantiation of the bare kernel name `kernel`."""
    return {k: v for k, v in kernel_hashes(lib_path, arch).items() if demangled_base(k) == kernel}


def base_hashes(lib_path, arch="gfx950"):
    """{bare kernel name: one sha256 over the hashes of all its instantiations} -- what profiles/ stamps on
    each PMC summary and bench.py compares against the library it times (any instantiation changing makes
    the summary stale)."""
    groups = {}
    for k, v in kernel_hashes(lib_path, arch).items():
        groups.setdefault(demangled_base(k), []).append(k + ":" + v)
    return {b: hashlib.sha256("\n".join(sorted(vs)).encode()).hexdigest() for b, vs in groups.items()}


def profile_kernel_base(name):
    """rocprofv3's demangled `prt::k_trace2<32, 9, 7, 64, false, false>` -> `k_trace2`."""
    return name.split("(")[0].replace("void ", "").strip().split("<")[0].split("::")[-1]


if __name__ == "__main__":  # python -m prt.codeobj [lib]: the bare-name hashes as JSON (written on the GPU box)
    import json
    import os
    import sys
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "libprt.so")
    print(json.dumps({"lib": os.path.basename(lib), "kernels": base_hashes(lib)}, indent=1, sort_keys=True))
