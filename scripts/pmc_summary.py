"""Summarise a rocprofv3 --pmc sqlite db: per kernel, mean duration and mean counters."""
import collections
import sqlite3
import sys


def summarise(path, top=4):
    c = sqlite3.connect(path)
    q = """select s.display_name, d.start, d.end, p.name, e.value, d.id
           from rocpd_kernel_dispatch d
           join rocpd_info_kernel_symbol s on s.id = d.kernel_id
           left join rocpd_pmc_event e on e.event_id = d.event_id
           left join rocpd_info_pmc p on p.id = e.pmc_id"""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for name, st, en, pname, val, did in c.execute(q):
        disp[name][did] = en - st
        if pname:
            per[name][pname] += val or 0.0
    rows = []
    for name, d in disp.items():
        n = len(d)
        rows.append((sum(d.values()) / n / 1e3, n, name, {k: v / n for k, v in per[name].items()}))
    rows.sort(key=lambda r: -r[0] * r[1])
    out = []
    for us, n, name, cnt in rows[:top]:
        out.append(f"{name[:90]}  n={n}  mean={us:.1f}us")
        wc = cnt.get("SQ_WAVE_CYCLES", 0)
        for k in sorted(cnt):
            extra = f"  ({100 * cnt[k] / wc:.1f}% of wave cycles)" if wc and k.startswith("SQ_WAIT") or (wc and k == "SQ_ACTIVE_INST_ANY") else ""
            out.append(f"    {k:28s} {cnt[k]:.4g}{extra}")
    return "\n".join(out)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        print("##", p)
        print(summarise(p))
