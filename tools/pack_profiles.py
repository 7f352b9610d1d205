"""Pack a round's per-run profile files into one markdown file.

    python tools/pack_profiles.py profiles/r04 [more dirs]

For every file under the directory (recursively) the pack holds a section headed by
its path relative to profiles/ -- a table row of the headline fields for a bench JSON
line, the file itself verbatim (text) below.  The originals can then be removed from
the tree; DESIGN.md cites `profiles/<dir>.md` § <relative path>.  Binary files are
skipped (and listed)."""
from __future__ import annotations

import json
import os
import sys


def headline(path):
    try:
        lines = [ln for ln in open(path).read().splitlines() if ln.strip().startswith("{")]
        d = json.loads(lines[-1])
    except Exception:
        return None
    if "value" not in d:
        return None
    r = d.get("roofline") or {}
    return (f"{d.get('value')}", f"{d.get('ms_per_step')}", f"{r.get('frac')}")


def pack(d):
    root = os.path.dirname(os.path.abspath(d))
    files = []
    for dp, _, fs in os.walk(d):
        for f in sorted(fs):
            files.append(os.path.join(dp, f))
    files.sort()
    out = [f"# {os.path.relpath(d, root)} -- packed run records", "",
           "Every file this directory held, verbatim (packed by tools/pack_profiles.py); sections are "
           "headed by the original path.", "", "| file | value | ms/step | roofline frac |", "|---|---|---|---|"]
    body, skipped = [], []
    for p in files:
        rel = os.path.relpath(p, root)
        try:
            txt = open(p, encoding="utf-8").read()
        except UnicodeDecodeError:
            skipped.append(rel)
            continue
        h = headline(p)
        if h:
            out.append(f"| {rel} | {h[0]} | {h[1]} | {h[2]} |")
        body += ["", f"## {rel}", "", "```", txt.rstrip("\n"), "```"]
    if skipped:
        out += ["", "Binary files not packed: " + ", ".join(skipped)]
    dest = os.path.abspath(d).rstrip("/") + ".md"
    with open(dest, "w") as f:
        f.write("\n".join(out + body) + "\n")
    print(dest, len(files), "files", os.path.getsize(dest), "bytes", "skipped", len(skipped))
    return skipped


if __name__ == "__main__":
    for d in sys.argv[1:]:
        pack(d)
