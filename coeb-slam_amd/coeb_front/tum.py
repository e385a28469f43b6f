"""TUM RGB-D timestamp association (the reference's associate.py, read_file_list + associate).

Host-side ingest: pairs rgb/depth (or groundtruth) time stamps
greedily by |t_a - (t_b + offset)| < max_difference, smallest difference first, each stamp
used once; ties broken by (difference, a, b) as the reference's sorted tuple list does.
"""


def read_file_list(text_or_path):
    """associate.py read_file_list: {stamp: [fields...]} from "stamp d1 d2 ..." lines
    (',' and tabs count as spaces, '#' lines skipped, lines with < 2 fields dropped)."""
    if "\n" not in text_or_path:
        with open(text_or_path) as f:
            text_or_path = f.read()
    lines = text_or_path.replace(",", " ").replace("\t", " ").split("\n")
    rows = [[v.strip() for v in line.split(" ") if v.strip() != ""] for line in lines
            if len(line) > 0 and line[0] != "#"]
    return dict((float(r[0]), r[1:]) for r in rows if len(r) > 1)


def associate(first, second, offset=0.0, max_difference=0.02):
    """associate.py associate: sorted list of matched (stamp_first, stamp_second)."""
    cand = sorted((abs(a - (b + offset)), a, b) for a in first for b in second
                  if abs(a - (b + offset)) < max_difference)
    fa, sb = set(first), set(second)
    out = []
    for _, a, b in cand:
        if a in fa and b in sb:
            fa.remove(a)
            sb.remove(b)
            out.append((a, b))
    out.sort()
    return out
