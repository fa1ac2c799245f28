"""Static checks over the gfx950 code objects of a built library (libpzkwit.so).

Check 1 — return address clobbered by long-branch expansion (the cause of the round-2 EC-walker hang /
fault). A callable (non-kernel) device function receives its return address in
s[30:31] and returns with `s_setpc_b64 s[30:31]`. When a function is larger than the ±128 KiB reach of
s_branch / s_cbranch, LLVM's branch relaxation expands far branches into
`s_getpc_b64 sX; s_add_u32 ...; s_addc_u32 ...; s_setpc_b64 sX` with a scavenged SGPR pair. The ROCm 7.2
compiler can pick s[30:31] for that pair in a function that did not save the return address first, and
the function then "returns" into its own body: an endless loop (the P-256 table walker) or a jump into
arbitrary code (an illegal memory access, the brainpool walker). A kernel has no return address, so only
non-kernel functions are checked: one whose body writes s30 / s31 (s_getpc, s_mov, s_add ...) and never
saves them (v_writelane of s30 / s31, or a copy of s[30:31]) before returning through s[30:31] fails.

Usage: python tools/check_code_objects.py [path/to/libpzkwit.so]   (exit 1 on a finding)
"""
import os
import re
import shutil
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def code_objects(lib, tmp):
    """gfx950 code objects bundled in the host library (one per translation unit)."""
    dst = os.path.join(tmp, os.path.basename(lib))
    shutil.copy(lib, dst)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", dst], check=True, capture_output=True)
    return sorted(os.path.join(tmp, f) for f in os.listdir(tmp) if "amdgcn-amd-amdhsa--gfx950" in f)


def functions(co):
    """(name, is_kernel, [instruction lines]) per function symbol of a code object."""
    syms = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "-sW", co], check=True, capture_output=True,
                          text=True).stdout
    kernels = {m.group(1)[:-3] for m in re.finditer(r"\bOBJECT\s+\S+\s+\S+\s+\S+\s+(\S+\.kd)\b", syms)}
    dis = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--no-show-raw-insn", "--no-leading-addr", co],
                         check=True, capture_output=True, text=True).stdout
    out, cur, body = [], None, []
    for line in dis.splitlines():
        m = re.match(r"^(?:[0-9a-f]+ )?<(\S+)>:\s*$", line)
        if m:
            if cur is not None:
                out.append((cur, cur in kernels, body))
            cur, body = m.group(1), []
        elif cur is not None and line.strip() and not line.strip().startswith(";"):
            body.append(line.split("//")[0].strip())
    if cur is not None:
        out.append((cur, cur in kernels, body))
    return out


WRITES_RA = re.compile(r"^(?!s_setpc|s_cmp|s_bitcmp)s_\w+\s+(s\[30:31\]|s30|s31)\s*(,|$)")
SAVES_RA = re.compile(r"^(v_writelane_b32\s+v\d+,\s*s3[01],|s_mov_b64\s+s\[\d+:\d+\],\s*s\[30:31\]|"
                      r"s_mov_b32\s+s\d+,\s*s3[01]$|scratch_store\w*\s.*s\[30:31\])")


def return_address_clobbers(body):
    """instructions that overwrite s30/s31 before any save of them, in a function returning via s[30:31]"""
    if not any(re.match(r"^s_setpc_b64\s+s\[30:31\]$", i) for i in body):
        return []
    bad = []
    for ins in body:
        if SAVES_RA.match(ins):
            return bad
        if WRITES_RA.match(ins):
            bad.append(ins)
    return bad


def check(lib):
    findings = []
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(lib, tmp):
            for name, is_kernel, body in functions(co):
                if is_kernel:
                    continue
                bad = return_address_clobbers(body)
                if bad:
                    findings.append("%s: %s (%d instructions, first: %s)" % (os.path.basename(co), name, len(body), bad[0]))
    return findings


if __name__ == "__main__":
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(here, "passport-zk-circuits_amd", "lib", "libpzkwit.so")
    f = check(lib)
    print("\n".join(f) if f else "ok: no callable function overwrites its return address before saving it")
    sys.exit(1 if f else 0)
