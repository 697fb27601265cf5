"""Build an A/B variant of liblsr.so from a patched COPY of csrc (the product
sources stay free of experiment switches).

    python tools/variant.py NAME 'old text' 'new text' [file.hip] [-- 'old2' 'new2' [file2]] ...
    python tools/variant.py NAME --patch tools/variants/X.patch [--patch ...] [-- 'old' 'new' ...]

Each replacement must match exactly once in its file (default render.hip).
Output: langsplatv2_amd/_build/var_NAME/liblsr.so (sources + objects under var_NAME/pkg) (load with tools/ab.py NAME=path)."""
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "langsplatv2_amd", "csrc")


def main():
    name = sys.argv[1]
    groups, cur = [], []
    for a in sys.argv[2:]:
        if a == "--":
            groups.append(cur)
            cur = []
        else:
            cur.append(a)
    if cur:
        groups.append(cur)
    dst = os.path.join(ROOT, "langsplatv2_amd", "_build", "var_" + name)
    src = os.path.join(dst, "pkg", "csrc")   # the same relative layout as langsplatv2_amd/csrc
    shutil.rmtree(dst, ignore_errors=True)
    shutil.copytree(CSRC, src)
    inc = os.path.join(dst, "include")
    shutil.copytree(os.path.join(ROOT, "include"), inc)
    for g in groups:
        if g and g[0] == "--patch":
            # a unified diff against langsplatv2_amd/csrc (a/langsplatv2_amd/csrc/<file>)
            for pf in g[1::2]:
                subprocess.run(["patch", "-s", "-p3", "-d", src, "-i", os.path.abspath(pf)], check=True)
            continue
        old, new = g[0], g[1]
        fn = g[2] if len(g) > 2 else "render.hip"
        p = os.path.join(src, fn)
        s = open(p).read()
        n = s.count(old)
        if n != 1:
            raise SystemExit(f"{fn}: pattern matches {n} times: {old[:80]!r}")
        open(p, "w").write(s.replace(old, new))
    subprocess.run(["make", "-s", "-j", "8", "-C", src], check=True)
    out = os.path.join(dst, "liblsr.so")
    shutil.move(os.path.join(dst, "pkg", "liblsr.so"), out)
    print(out)


if __name__ == "__main__":
    main()
