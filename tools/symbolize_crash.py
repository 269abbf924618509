"""Resolve the "(unknown)" frames of a crash log that carries a PPO_SEGV_MAPS=1 maps dump
(csrc/host/crash_maps.c): every "@ 0x..." stack address and the faulting address are matched
against /proc/self/maps as it was at the fault, reported as library + offset and symbolised with
llvm-symbolizer (module-relative addresses: the library's base is the start of its offset-0
mapping).  Usage: python tools/symbolize_crash.py <crash log> [out.txt]
"""
import re
import subprocess
import sys

SYMBOLIZER = "/opt/rocm/llvm/bin/llvm-symbolizer"


def parse(text):
    maps, in_maps = [], False
    for line in text.splitlines():
        if line.startswith("--- /proc/self/maps"):
            in_maps = True
            continue
        if line.startswith("--- end maps"):
            in_maps = False
            continue
        if in_maps:
            m = re.match(r"([0-9a-f]+)-([0-9a-f]+) (\S+) ([0-9a-f]+) \S+ \d+\s*(.*)", line)
            if m:
                maps.append((int(m[1], 16), int(m[2], 16), m[3], int(m[4], 16), m[5].strip()))
    frames = [int(a, 16) for a in re.findall(r"@\s+(0x[0-9a-f]+)", text)]
    fault = re.search(r"crash_maps: signal \S+ at address (0x[0-9a-f]+)", text)
    return maps, frames, int(fault[1], 16) if fault else None


def where(maps, addr):
    for lo, hi, perm, off, path in maps:
        if lo <= addr < hi:
            base = min((l for l, _, _, o, p in maps if p == path and o == 0), default=lo)
            return lo, hi, perm, off, path, base
    return None


def symbolize(path, rel):
    if not path.startswith("/"):
        return ""
    try:
        out = subprocess.run([SYMBOLIZER, f"--obj={path}", hex(rel), "--demangle"],
                             capture_output=True, text=True, timeout=60).stdout.strip()
        return " | ".join(x for x in out.splitlines() if x)
    except Exception as e:  # symbolizer missing / timeout
        return f"(symbolizer: {e})"


def main():
    text = open(sys.argv[1], errors="replace").read()
    maps, frames, fault = parse(text)
    lines = []
    if fault is not None:
        w = where(maps, fault)
        lines.append(f"fault address {fault:#x}: " + (
            f"inside {w[4] or '[anon]'} [{w[0]:#x}-{w[1]:#x} {w[2]} off {w[3]:#x}]" if w else
            "in NO mapping"))
        below = [m for m in maps if m[1] <= fault]
        above = [m for m in maps if m[0] > fault]
        if below:
            m = max(below, key=lambda x: x[1])
            lines.append(f"  mapping ending at/below it: {m[0]:#x}-{m[1]:#x} {m[2]} {m[4] or '[anon]'} "
                         f"({fault - m[1]:#x} bytes past its end)")
        if above:
            m = min(above, key=lambda x: x[0])
            lines.append(f"  next mapping above it: {m[0]:#x}-{m[1]:#x} {m[2]} {m[4] or '[anon]'}")
    for a in frames:
        w = where(maps, a)
        if not w:
            lines.append(f"{a:#x}  (no mapping)")
            continue
        lo, hi, perm, off, path, base = w
        rel = a - base
        lines.append(f"{a:#x}  {path or '[anon]'} +{rel:#x}  {symbolize(path, rel)}")
    out = "\n".join(lines)
    print(out)
    if len(sys.argv) > 2:
        open(sys.argv[2], "w").write(out + "\n")


if __name__ == "__main__":
    main()
