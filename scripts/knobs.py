"""List every MLOP_* environment variable the code reads (name, default, file:line).

    python scripts/knobs.py            # print the table body (used to write docs/KNOBS.md)
    python scripts/knobs.py --check    # exit 1 if a knob read in the code is missing from docs/KNOBS.md
"""
import re
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "research-and-development-of-kubernetes-operator-for-machine-learning-pipelines_amd"
PATS = [
    re.compile(r'os\.environ\.get\(\s*"(MLOP_[A-Z0-9_]+)"\s*(?:,\s*([^)]*?))?\)'),
    re.compile(r'os\.environ\[\s*"(MLOP_[A-Z0-9_]+)"\s*\]()'),
    re.compile(r'os\.getenv\(\s*"(MLOP_[A-Z0-9_]+)"\s*(?:,\s*([^)]*?))?\)'),
    re.compile(r'(?<![A-Za-z_])getenv\(\s*"(MLOP_[A-Z0-9_]+)"\s*\)()'),
    re.compile(r'env_int\(\s*"(MLOP_[A-Z0-9_]+)"\s*,\s*([^)]*?)\)'),
    re.compile(r'"(MLOP_[A-Z0-9_]+)"\s+in\s+os\.environ()'),
    re.compile(r'(?<![A-Za-z_])e\.get\(\s*"(MLOP_[A-Z0-9_]+)"\s*,\s*([^)]*?)\)'),  # OperatorSettings.from_env
]


def scan():
    found = {}
    files = [ROOT / "bench.py", ROOT / "__graft_entry__.py"]
    for ext in ("*.py", "*.hip", "*.cpp", "*.h"):
        files += sorted(PKG.rglob(ext))
    for f in files:
        if "__pycache__" in f.parts or "_build" in f.parts:
            continue
        for i, line in enumerate(f.read_text().splitlines(), 1):
            for p in PATS:
                for m in p.finditer(line):
                    name, dflt = m.group(1), (m.group(2) or "").strip()
                    e = found.setdefault(name, {"default": "", "where": []})
                    if dflt and not e["default"]:
                        e["default"] = dflt
                    e["where"].append(f"{f.relative_to(ROOT)}:{i}")
    return found


def main():
    found = scan()
    if "--check" in sys.argv:
        doc = (ROOT / "docs" / "KNOBS.md").read_text()
        missing = [n for n in found if f"`{n}`" not in doc]
        # and the reverse: a documented knob nothing reads any more (a removed A/B switch)
        import re

        documented = {m for row in doc.splitlines() if row.startswith("| `MLOP_")
                      for m in re.findall(r"`(MLOP_[A-Z0-9_]+)`", row.split("|")[1])}
        stale = sorted(n for n in documented if n not in found and not n.startswith("MLOP_ENGINE_"))
        if missing:
            print("not in docs/KNOBS.md:", ", ".join(sorted(missing)))
        if stale:
            print("documented but read nowhere:", ", ".join(stale))
        return 1 if (missing or stale) else 0
    for name in sorted(found):
        e = found[name]
        print(f"| `{name}` | {e['default'] or '—'} | {', '.join(e['where'][:2])} |")
    return 0


if __name__ == "__main__":
    sys.exit(main())
