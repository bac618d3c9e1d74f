"""Static ISA budget of a kernel by source phase (round 6).

Compiles a csrc/*.hip file for gfx950 with line tables (-gline-tables-only, same flags as
the Makefile), takes one kernel's body from the assembly and attributes every instruction
to the phase of the source line it came from.  Phases are marked in the source by comments
`// phase: NAME` (the phase holds until the next marker, in the kernel and in the device
functions it calls); instructions from other files (det.h, the HIP headers) count for the
phase of the last line of the source file seen before them.

    python tools/isa_budget.py scan_batches.hip 'k_scan_batches_classifyILb0ELi7' [--json out]

Static counts: every instruction of the kernel once, whichever branch it is on; the dynamic
count per fill comes from SQ_INSTS_VALU (rocprofv3 --pmc) over the fills of a call."""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

CSRC = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "distributed-drift-detection_amd", "csrc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off", "-fno-fast-math",
         "-mcode-object-version=5", "-gline-tables-only", "--offload-device-only", "-S"]


def phases_of(src_lines):
    ph, out = "other", {}
    for i, l in enumerate(src_lines, 1):
        m = re.search(r"//\s*phase:\s*([\w/+-]+)", l)
        if m:
            ph = m.group(1)
        out[i] = ph
    return out


def kinds(ins):
    op = ins.split()[0]
    if op.startswith("v_"):
        return "valu"
    if op.startswith("s_"):
        return "salu" if not op.startswith(("s_waitcnt", "s_nop", "s_barrier", "s_cbranch", "s_branch",
                                            "s_load", "s_buffer", "s_endpgm", "s_sleep", "s_setprio")) else "sctl"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    return "other"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("kernel", help="substring of the mangled kernel name")
    ap.add_argument("--json")
    ap.add_argument("--defines", nargs="*", default=[])
    a = ap.parse_args()
    src = a.src
    out = "/tmp/isa_budget.s"
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *["-D" + d for d in a.defines], a.src, "-o", out], check=True,
                   cwd=CSRC, stderr=subprocess.DEVNULL)
    asm = open(out).read().splitlines()
    files = {}
    for l in asm:
        m = re.match(r'\s*\.file\s+(\d+)\s+"[^"]*"\s+"([^"]+)"', l)
        if m:
            files[int(m.group(1))] = m.group(2)
    main_id = [k for k, v in files.items() if os.path.basename(v) == os.path.basename(a.src)][0]
    phase = phases_of(open(os.path.join(CSRC, a.src)).read().splitlines())
    start = next(i for i, l in enumerate(asm) if re.match(r"^_Z\S*%s\S*:(\s*;.*)?$" % re.escape(a.kernel), l))
    cnt = collections.defaultdict(collections.Counter)
    cur = "other"
    total = collections.Counter()
    for l in asm[start + 1:]:
        s = l.strip()
        if s.startswith(".Lfunc_end"):
            break
        m = re.match(r"\.loc\s+(\d+)\s+(\d+)", s)
        if m:
            if int(m.group(1)) == main_id and int(m.group(2)) > 0:
                cur = phase.get(int(m.group(2)), "other")
            continue
        if not s or s.startswith((".", ";", "/")) or s.endswith(":"):
            continue
        k = kinds(s)
        cnt[cur][k] += 1
        total[k] += 1
    rows = {p: dict(c) for p, c in sorted(cnt.items(), key=lambda x: -x[1]["valu"])}
    print(f"{'phase':<16}" + "".join(f"{k:>7}" for k in ("valu", "salu", "lds", "vmem", "sctl")))
    for p, c in rows.items():
        print(f"{p:<16}" + "".join(f"{c.get(k, 0):>7}" for k in ("valu", "salu", "lds", "vmem", "sctl")))
    print(f"{'TOTAL':<16}" + "".join(f"{total.get(k, 0):>7}" for k in ("valu", "salu", "lds", "vmem", "sctl")))
    if a.json:
        json.dump({"kernel": a.kernel, "src": a.src, "static": rows, "total": dict(total)}, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    sys.exit(main())
