"""Instruction mix of the innermost loops of a kernel in a hipcc .s file
(blocks LLVM annotates as belonging to the loop).
Usage: python tools/loop_stats.py FILE.s KERNEL_SYMBOL"""
import collections
import re
import sys


def main():
    path, sym = sys.argv[1], sys.argv[2]
    txt = open(path).read().split("\n")
    s = next(i for i, l in enumerate(txt) if l.startswith(sym + ":"))
    e = next(i for i in range(s, len(txt)) if txt[i].startswith(".Lfunc_end"))
    lines = txt[s:e + 1]
    blocks, cur = {}, None
    for i, l in enumerate(lines):
        if l.startswith(".LBB") or l.startswith("; %bb."):
            cur = l.split(":")[0].split()[-1] if l.startswith(".") else l.split()[1].rstrip(":")
            hdr = re.search(r"Header=(\S+) Depth=(\d+)", l)
            nxt = lines[i + 1] if i + 1 < len(lines) else ""
            if "Inner Loop Header" in nxt or "Loop Header" in nxt:
                d = re.search(r"Depth=(\d+)", nxt)
                blocks[cur] = dict(loop=cur.lstrip(".").replace("LBB", "BB"), depth=int(d.group(1)) if d else 0, ins=[])
            elif hdr:
                blocks[cur] = dict(loop=hdr.group(1), depth=int(hdr.group(2)), ins=[])
            else:
                blocks[cur] = dict(loop=None, depth=0, ins=[])
            continue
        x = l.strip()
        if cur and x and not x.startswith(";") and not x.startswith("."):
            blocks[cur]["ins"].append(x.split()[0])
    loops = collections.defaultdict(list)
    for b in blocks.values():
        if b["loop"]:
            loops[(b["loop"], b["depth"])].append(b["ins"])
    for (lp, d), ins in sorted(loops.items(), key=lambda t: -t[0][1]):
        cat = collections.Counter()
        for blk in ins:
            for op in blk:
                cat["valu" if op.startswith("v_") else "salu" if op.startswith("s_") else "lds" if op.startswith(
                    "ds_") else "vmem" if op.startswith(("global_", "buffer_")) else op] += 1
        print(f"loop {lp} depth {d}: {sum(cat.values())} instructions {dict(cat)}")


if __name__ == "__main__":
    main()
