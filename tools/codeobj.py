"""Read the gfx950 code objects embedded in librtow_hip.so.

The .hip_fatbin section holds one clang offload bundle per HIP translation
unit (magic "__CLANG_OFFLOAD_BUNDLE__", then entry count and per entry:
offset, size, triple).  For every kernel of every gfx950 code object this
returns what the code-object metadata records (VGPRs, SGPRs, scratch bytes
per lane, spill counts, dynamic stack, LDS) and whether the kernel's code
contains a call (s_swappc_b64, or an s_setpc_b64 that is not a long branch
within the kernel): the shipped binary itself, not
a recompilation.  Used by tests/test_build_resources.py.

  python tools/codeobj.py [path/to/librtow_hip.so]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def fatbin_section(path):
    data = open(path, "rb").read()
    out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-S", "-W", path], capture_output=True, text=True,
                         check=True).stdout
    for line in out.splitlines():
        if ".hip_fatbin" in line:
            f = line.split("]", 1)[1].split()
            off, size = int(f[3], 16), int(f[4], 16)
            return data[off:off + size]
    raise RuntimeError(f"{path}: no .hip_fatbin section")


def code_objects(path, arch="gfx950"):
    """The ELF code objects for `arch` in the library's fat binary."""
    sec = fatbin_section(path)
    objs = []
    pos = sec.find(MAGIC)
    while pos >= 0:
        (n,) = struct.unpack_from("<Q", sec, pos + 24)
        p = pos + 32
        end = pos
        for _ in range(n):
            off, size, tlen = struct.unpack_from("<QQQ", sec, p)
            triple = sec[p + 24:p + 24 + tlen].decode()
            p += 24 + tlen
            if arch in triple and size:
                objs.append(sec[pos + off:pos + off + size])
            end = max(end, pos + off + size)
        pos = sec.find(MAGIC, max(end, pos + 1))
    return objs


def _kernel_metadata(elf_path):
    """Per-kernel records of the NT_AMDGPU_METADATA note: the kernel-level
    keys of each `amdhsa.kernels` entry (indentation 4 in llvm-readelf's dump;
    the argument list nests deeper), keyed by the kernel's .name."""
    out = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", elf_path], capture_output=True, text=True,
                         check=True).stdout
    recs, cur = [], None
    for line in out.splitlines():
        m = re.match(r"^  - \.(\w+):\s*(.*)$", line)
        if m:
            cur = {m.group(1): m.group(2).strip()}
            recs.append(cur)
            continue
        m = re.match(r"^    \.(\w+):\s*(.*)$", line)
        if m and cur is not None:
            cur[m.group(1)] = m.group(2).strip()
        elif re.match(r"^\S", line) or line.startswith("amdhsa.target"):
            cur = None
    return {r["name"]: r for r in recs if "name" in r}


def kernels(path):
    """[{name, vgpr, sgpr, scratch, vgpr_spill, sgpr_spill, dyn_stack, lds, calls}] over all code objects."""
    res = []
    for obj in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(obj)
            co = f.name
        try:
            meta = _kernel_metadata(co)
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                                 capture_output=True, text=True, check=True).stdout
        finally:
            os.unlink(co)
        calls, cur = {}, None
        lines = dis.splitlines()
        for i, line in enumerate(lines):
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                cur = m.group(1)
                calls.setdefault(cur, 0)
            elif cur and re.search(r"\bs_swappc_b64\b", line):
                calls[cur] += 1
            elif cur and re.search(r"\bs_setpc_b64\b", line):
                # a long branch inside a huge kernel is s_getpc_b64 s[a:b];
                # s_add_u32 sa, sa, off; s_addc_u32 sb, sb, 0; s_setpc_b64 s[a:b]
                # (same function, target computed from its own pc): not a call
                reg = re.search(r"s_setpc_b64\s+(s\[\d+:\d+\])", line)
                prev = " ".join(lines[max(0, i - 4):i])
                if not (reg and re.search(r"s_getpc_b64\s+" + re.escape(reg.group(1)), prev)):
                    calls[cur] += 1
        for name, m in meta.items():
            res.append({"name": name, "vgpr": int(m.get("vgpr_count", -1)), "sgpr": int(m.get("sgpr_count", -1)),
                        "scratch": int(m.get("private_segment_fixed_size", -1)),
                        "vgpr_spill": int(m.get("vgpr_spill_count", 0)), "sgpr_spill": int(m.get("sgpr_spill_count", 0)),
                        "dyn_stack": m.get("uses_dynamic_stack", "false") == "true",
                        "lds": int(m.get("group_segment_fixed_size", 0)),
                        "calls": calls.get(name, 0),
                        # code symbols of this object that are not kernels: out-of-line device functions
                        "functions": sorted(k for k in calls if k not in meta and not k.startswith("__"))})
    return res


def demangled_params(name):
    """trace_kernel<MODE, STACK, WAVES, PROF, BS, LDSN, DBG> template values."""
    m = re.search(r"trace_kernelILi(\d+)ELi(\d+)ELi(\d+)ELb(\d)ELi(\d+)ELb(\d)ELb(\d)E", name)
    if not m:
        return None
    keys = ("MODE", "STACK", "WAVES", "PROF", "BS", "LDSN", "DBG")
    return dict(zip(keys, (int(v) for v in m.groups())))


def disasm(path, want):
    """The disassembly (text) of the kernel whose demangled template
    parameters equal `want` (a dict, e.g. {"MODE": 8, "STACK": 16, "WAVES": 4,
    "PROF": 0, "BS": 256, "LDSN": 0, "DBG": 0})."""
    for obj in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(obj)
            co = f.name
        try:
            meta = _kernel_metadata(co)
            names = [n for n in meta if demangled_params(n) == want]
            if not names:
                continue
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                                 capture_output=True, text=True, check=True).stdout
        finally:
            os.unlink(co)
        out, on = [], False
        for line in dis.splitlines():
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                on = m.group(1) == names[0]
            if on:
                out.append(line)
        return "\n".join(out)
    return None


def isa_digest(path):
    """{kernel symbol: sha256 of its disassembly with addresses stripped} over
    every code object: two builds whose digests agree run the same machine
    code (used to check that a host-side refactor leaves the kernels alone)."""
    import hashlib

    res = {}
    for obj in code_objects(path):
        with tempfile.NamedTemporaryFile(suffix=".co", delete=False) as f:
            f.write(obj)
            co = f.name
        try:
            dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", co],
                                 capture_output=True, text=True, check=True).stdout
        finally:
            os.unlink(co)
        cur, body = None, []
        for line in dis.splitlines() + ["0 <__end__>:"]:
            m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
            if m:
                if cur is not None:
                    res[cur] = hashlib.sha256("\n".join(body).encode()).hexdigest()[:16]
                cur, body = m.group(1), []
            elif cur is not None and line.strip():
                # drop the address column and branch-target addresses, keep the instruction
                body.append(re.sub(r"<[^>]*>|\b0x[0-9a-f]+\b", "", line.split("//")[0]).strip())
    return res


if __name__ == "__main__":
    # python tools/codeobj.py [LIB]                           : every kernel's resources
    # python tools/codeobj.py LIB MODE STACK [WAVES BS LDSN] > kernel.s : one kernel's disassembly
    a = sys.argv
    lib = a[1] if len(a) > 1 else os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                               "ray-tracing-one-weekend_amd", "librtow_hip.so")
    if len(a) > 2 and a[2] == "--digest":
        for name, h in sorted(isa_digest(lib).items()):
            print(h, name)
        sys.exit(0)
    if len(a) > 2:
        want = {"MODE": int(a[2]), "STACK": int(a[3]), "WAVES": int(a[4]) if len(a) > 4 else 4, "PROF": 0,
                "BS": int(a[5]) if len(a) > 5 else 256, "LDSN": int(a[6]) if len(a) > 6 else 0, "DBG": 0}
        print(disasm(lib, want))
    else:
        for k in kernels(lib):
            p = demangled_params(k["name"])
            print(p or k["name"][:40], {x: k[x] for x in ("vgpr", "scratch", "vgpr_spill", "sgpr_spill", "dyn_stack",
                                                           "lds", "calls")})
