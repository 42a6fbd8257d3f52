"""Where a config-2 step's wall time goes on the device, from a rocprofv3 CSV kernel trace (tools/gpu_r05.sh trace):
the union of all kernel intervals (device busy), the gaps in which no kernel runs (waiting on the host), and per
kernel family the time in which it is the only kernel running.  Usage: python3 tools/gpu_idle.py <trace dir>"""
import csv
import os
import sys


def main(d):
    rows = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("uc::", "")
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name.split("<")[0]))
    rows.sort()
    # the timed region: from the first counting launch after the warm-up's last traceback
    tw = [i for i, r in enumerate(rows) if r[2] == "k_trace_wave"]
    i0 = tw[1] + 1 if len(tw) > 2 else 0  # warm-up's two traceback launches (<= 64 nt and longer)
    rows = rows[i0:]
    t0, t1 = rows[0][0], max(r[1] for r in rows)
    busy, cur_s, cur_e = 0, rows[0][0], rows[0][1]
    gaps = []
    for s, e, _ in rows[1:]:
        if s > cur_e:
            busy += cur_e - cur_s
            gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    # sole-running time per family: sweep events
    ev = []
    for s, e, n in rows:
        ev.append((s, 1, n))
        ev.append((e, -1, n))
    ev.sort(key=lambda x: (x[0], x[1]))
    live, sole, last = {}, {}, ev[0][0]
    for t, k, n in ev:
        if len(live) == 1:
            only = next(iter(live))
            sole[only] = sole.get(only, 0) + (t - last)
        last = t
        live[n] = live.get(n, 0) + k
        if live[n] == 0:
            del live[n]
    wall = t1 - t0
    gaps.sort(reverse=True)
    print(f"window {wall / 1e6:.1f} ms, device busy {busy / 1e6:.1f} ms ({busy / wall:.3f}), idle {(wall - busy) / 1e6:.1f} ms "
          f"in {len(gaps)} gaps (largest {', '.join(f'{g / 1e3:.0f}' for g in gaps[:8])} us)")
    for n, t in sorted(sole.items(), key=lambda x: -x[1])[:12]:
        print(f"  sole {n:24s} {t / 1e6:8.1f} ms")


if __name__ == "__main__":
    main(sys.argv[1])
