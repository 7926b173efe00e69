"""Phase breakdown of tools/e2e_trace.py's rocprofv3 HIP API + kernel + copy
trace: per marked phase (hipRuntimeGetVersion markers: open, build, close), the
wall time, the HIP API calls by total duration, the kernels' and copies' busy
time, and the host time not inside any HIP call.

  python3 tools/api_timeline.py gpurun_out/TAG/trace [rep]"""
import collections
import csv
import glob
import os
import sys


def rows(d, suffix):
    out = []
    for p in glob.glob(os.path.join(d, "**", f"*{suffix}"), recursive=True):
        out += list(csv.DictReader(open(p)))
    return out


def busy(iv):
    """total length of the union of intervals"""
    t, end = 0, None
    for a, b in sorted(iv):
        if end is None or a > end:
            t += b - a
            end = b
        elif b > end:
            t += b - end
            end = b
    return t


def main() -> None:
    d = sys.argv[1]
    api = rows(d, "hip_api_trace.csv")
    kern = rows(d, "kernel_trace.csv")
    copy = rows(d, "memory_copy_trace.csv")
    for r in api + kern + copy:
        r["a"], r["b"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    api.sort(key=lambda r: r["a"])
    marks = [r["a"] for r in api if r["Function"] == "hipRuntimeGetVersion"]
    # the trace script's markers come in threes per rep (open, build, close),
    # the last one ends where the trace ends
    marks = marks[-9:]
    end = max(r["b"] for r in api)
    names = ["open", "build", "close"]
    for rep in range(len(marks) // 3):
        print(f"== rep {rep}")
        for i in range(3):
            a = marks[3 * rep + i]
            b = marks[3 * rep + i + 1] if 3 * rep + i + 1 < len(marks) else end
            inside = [r for r in api if a <= r["a"] < b and r["Function"] != "hipRuntimeGetVersion"]
            tid = collections.Counter(r["Thread_Id"] for r in inside).most_common(1)
            main_tid = tid[0][0] if tid else None
            per = collections.defaultdict(lambda: [0, 0])
            for r in inside:
                per[r["Function"]][0] += r["b"] - r["a"]
                per[r["Function"]][1] += 1
            main_api = busy([(r["a"], r["b"]) for r in inside if r["Thread_Id"] == main_tid])
            k = [(r["a"], r["b"]) for r in kern if a <= r["a"] < b]
            c = [(r["a"], r["b"]) for r in copy if a <= r["a"] < b]
            print(f"  {names[i]:6s} wall {(b - a) / 1e6:8.3f} ms  main-thread HIP calls {main_api / 1e6:7.3f} ms  "
                  f"kernels busy {busy(k) / 1e6:6.3f} ms ({len(k)})  copies busy {busy(c) / 1e6:6.3f} ms ({len(c)})")
            for f, (t, n) in sorted(per.items(), key=lambda kv: -kv[1][0])[:12]:
                print(f"      {f:40s} {t / 1e6:8.3f} ms  x{n}")
            if k:
                first = min(x[0] for x in k)
                print(f"      first kernel at +{(first - a) / 1e6:.3f} ms, last kernel end +{(max(x[1] for x in k) - a) / 1e6:.3f} ms")


if __name__ == "__main__":
    main()
