"""Minimal stand-in for python-fire's flag syntax used by run_1d.sh / run_2d.sh:
`-equation='poisson_2d-sin_sin' -kernel='Matern52_Cos_1d' -nepoch=100000` (also `--k=v`,
`-k v`).  Values are parsed as int / float / bool where possible, else kept as strings."""


def _value(s):
    s = s.strip().strip("'\"")
    for conv in (int, float):
        try:
            return conv(s)
        except ValueError:
            pass
    if s in ("True", "False"):
        return s == "True"
    return s


def parse_flags(argv):
    out = {}
    i = 0
    while i < len(argv):
        a = argv[i]
        if not a.startswith("-"):
            raise SystemExit("unexpected argument: %s" % a)
        key = a.lstrip("-")
        if "=" in key:
            key, val = key.split("=", 1)
        elif i + 1 < len(argv) and not argv[i + 1].startswith("-"):
            i += 1
            val = argv[i]
        else:
            val = "True"
        out[key.replace("-", "_")] = _value(val)
        i += 1
    return out
