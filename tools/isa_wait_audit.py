"""ISA audit (round 6): which kernels wait for their global loads one at a time.

hipcc inserts `s_waitcnt vmcnt(N)` from a conservative count: a load guarded per element
(`ok ? p[i] : 0`, `if (ok) load(...)`) becomes a branch around the load, and at every join the
count falls back to vmcnt(0) — every load of a batch is then waited for before the next one is
issued. This compiles a source file to gfx950 assembly and, per kernel, counts the global loads
and the vmcnt(0) waits that follow a load within a few instructions (the serialisation
signature); `--seq NAME` prints a kernel's load / wait / barrier / branch sequence.
    python tools/isa_wait_audit.py recommender_amd/csrc/sort.hip [--top 15] [--seq MANGLED]"""
import argparse
import re
import subprocess
import sys
import tempfile
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def compile_s(src: str) -> str:
    out = Path(tempfile.mkdtemp()) / "k.s"
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
           "-munsafe-fp-atomics", f"-I{ROOT / 'include'}", "--cuda-device-only", "-S", src, "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode:
        sys.exit(r.stderr)
    return out.read_text()


def bodies(s: str):
    for name in re.findall(r"^(_Z[^\s:]+):", s, re.M):
        i = s.index(name + ":")
        j = s.find(".Lfunc_end", i)
        if j > 0:
            yield name, s[i:j].splitlines()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--seq", default=None)
    a = ap.parse_args()
    s = compile_s(a.src)
    if a.seq:
        for name, body in bodies(s):
            if name != a.seq:
                continue
            seq = []
            for line in body:
                t = line.strip()
                if t.startswith(("global_load", "global_store", "global_atomic")):
                    seq.append(t.split()[0].replace("global_", ""))
                elif "vmcnt" in t:
                    seq.append("W" + re.search(r"vmcnt\((\d+)\)", t).group(1))
                elif "Loop Header" in t:
                    seq.append("|loop|")
                elif "s_barrier" in t:
                    seq.append("BAR")
            print(" ".join(seq))
        return
    res = []
    for name, body in bodies(s):
        loads, ser, last = 0, 0, -100
        for k, line in enumerate(body):
            t = line.strip()
            if t.startswith(("global_load", "buffer_load")):
                loads, last = loads + 1, k
            elif "s_waitcnt vmcnt(0)" in t and k - last < 6:
                ser += 1
        if loads:
            res.append((ser, loads, name))
    for ser, loads, name in sorted(res, reverse=True)[:a.top]:
        dn = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
        print(f"{ser:4d} waits right behind a load / {loads:4d} loads  {dn[:100]}")


if __name__ == "__main__":
    main()
