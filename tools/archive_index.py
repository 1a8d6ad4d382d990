#!/usr/bin/env python3
"""Write profiles/archive/INDEX.md: the superseded evidence, grouped by pass tag (the file-name
prefix r<round><pass>), one line per tag listing its files.  usage: python tools/archive_index.py"""
import collections
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ARCH = os.path.join(ROOT, "profiles", "archive")


def main():
    groups = collections.OrderedDict()
    for f in sorted(os.listdir(ARCH)):
        if f == "INDEX.md":
            continue
        m = re.match(r"(r\d+[a-z]*)_(.*)", f)
        tag, rest = (m.group(1), m.group(2)) if m else ("other", f)
        groups.setdefault(tag, []).append(rest)
    lines = ["# profiles/archive",
             "",
             "Logs and profiles of passes superseded by later ones (the current evidence is at the top of",
             "`profiles/`, cited from DESIGN.md).  Kept for the history of the numbers DESIGN's tables quote;",
             "each line is one pass tag (round number + pass letter) and the files it left.",
             ""]
    def key(tag):
        m = re.match(r"r(\d+)([a-z]*)", tag)
        return (int(m.group(1)), len(m.group(2)), m.group(2)) if m else (99, 0, tag)
    for tag in sorted(groups, key=key):
        lines.append("* **%s** (%d): %s" % (tag, len(groups[tag]), ", ".join(groups[tag])))
    with open(os.path.join(ARCH, "INDEX.md"), "w") as fh:
        fh.write("\n".join(lines) + "\n")


if __name__ == "__main__":
    main()
