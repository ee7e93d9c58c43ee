"""Instruction mix of one kernel's basic blocks in a hipcc -S listing (quick ISA review).

    python tools/isa_mix.py file.s k_bp [--min 40]
"""
import collections
import re
import sys


def main():
    path, kern = sys.argv[1], sys.argv[2]
    mn = int(sys.argv[sys.argv.index("--min") + 1]) if "--min" in sys.argv else 40
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + kern + r"\S*:", l))
    end = next(i for i in range(start, len(lines)) if lines[i].strip().startswith(".Lfunc_end"))
    blocks, cur = [], ["entry", "", []]
    blocks.append(cur)
    for l in lines[start + 1:end]:
        m = re.match(r"^(\.LBB\d+_\d+):(.*)", l)
        if m:
            cur = [m.group(1), m.group(2).strip(), []]
            blocks.append(cur)
            continue
        s = l.strip()
        if not s or s.startswith(";") or s.startswith("."):
            continue
        cur[2].append(s.split()[0])
    tot = collections.Counter()
    for name, c, ins in blocks:
        cnt = collections.Counter()
        for i in ins:
            if i.startswith("v_"):
                k = "valu_f64" if "f64" in i else "valu"
            elif i.startswith("ds_"):
                k = "ds"
            elif i.startswith("s_"):
                k = "salu"
            elif "scratch" in i or "buffer" in i:
                k = "scratch"
            else:
                k = "other"
            cnt[k] += 1
        tot.update(cnt)
        if len(ins) >= mn:
            print(f"{name:12s} {c[:36]:36s} {len(ins):5d} {dict(cnt)}")
    print("total", dict(tot))


if __name__ == "__main__":
    main()


def loop_total(path, kern, header):
    """Sum of the instruction classes of a loop's blocks (header + blocks 'in Loop: Header=...')."""
    import subprocess
    out = subprocess.run([sys.executable, __file__, path, kern, "--min", "0"], capture_output=True, text=True).stdout
    tot = collections.Counter()
    for l in out.splitlines():
        if l.startswith("." + header[2:] if False else "") and (l.split()[0] == "." + header or f"Header={header}" in l):
            d = eval(l[l.index("{"):])
            tot.update(d)
    return dict(tot)
