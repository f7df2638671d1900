"""Summarise a rocprofv3 --kernel-trace CSV: per-step time by kernel family.
Usage: python tools/prof_summary.py <prof_dir> <num_steps_in_trace>"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def family(name: str) -> str:
    n = name
    m = re.search(r"conv_gemm_kernel<(\d+), (\d+), (\d+), (\d+)(?:, (\d+))?(?:, (\d+))?>", n) or \
        re.search(r"conv_gemm_kernelILi(\d+)ELi(\d+)ELi(\d+)ELi(\d+)E(?:Li(\d+)E)?(?:Li(\d+)E)?", n)
    if m:
        p = {"0": "fwd", "1": "dgrad", "2": "wgrad", "3": "wgrad_bna", "4": "dgrad_bnf",
             "5": "wgrad_gram", "6": "fwd_tail"}[m.group(1)]
        st = f" st{m.group(5)}" if m.group(5) else ""
        pro = " mf32" if m.group(6) == "32" else ""
        return f"conv_{p} {m.group(3)}x{m.group(4)}{st}{pro}"
    n = re.sub(r"^void ", "", n)
    n = n.replace("(anonymous namespace)::", "")
    if n.startswith("at::native::"):
        m = re.search(r"at::native::(\w+)<[^,]*, ([\w:]+)", n)
        return "aten " + (m.group(2).split("::")[-1] if m else n[12:40])
    n = re.sub(r"[<(].*", "", n)
    return n[:60]


def main():
    d = sys.argv[1]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    files = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not files:
        print("no kernel_trace.csv under", d)
        return
    rows = list(csv.DictReader(open(files[0])))
    # restrict to whole training steps: a step starts with its batch generation (synth*_kernel)
    # and its last kernel precedes the next step's generation; model construction (weight
    # copies, fills) and the bench's extra passes fall outside the window
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows)
              if re.match(r"(void )?(\(anonymous namespace\)::)?synth(_s2d)?_kernel",
                          (r.get("Kernel_Name") or r.get("KernelName") or ""))]
    if len(starts) >= 2:
        rows = rows[starts[0]:starts[-1]]      # steps 1 .. n-1 of the trace (the last may be partial)
        steps = len(starts) - 1
    tot = defaultdict(float)
    cnt = defaultdict(int)
    for r in rows:
        name = r.get("Kernel_Name") or r.get("KernelName") or ""
        t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        f = family(name)
        tot[f] += t
        cnt[f] += 1
    all_ms = sum(tot.values())
    print(f"# rocprofv3 kernel summary ({files[0].split('/')[-1]})\n")
    print(f"total GPU kernel time {all_ms:.2f} ms over {steps} steps = {all_ms / steps:.2f} ms/step\n")
    print("| kernel family | ms/step | % | launches/step |")
    print("|---|---|---|---|")
    for f, t in sorted(tot.items(), key=lambda kv: -kv[1]):
        print(f"| {f} | {t / steps:.3f} | {100 * t / all_ms:.1f} | {cnt[f] / steps:.1f} |")
    # device occupancy over the trace's last `steps` steps' window: union of kernel intervals
    # (kernels of the main and wgrad streams overlap) vs the wall span, and the idle gaps
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows)
    busy, gaps, cur_s, cur_e = 0, [], iv[0][0], iv[0][1]
    for s_, e_ in iv[1:]:
        if s_ > cur_e:
            busy += cur_e - cur_s
            gaps.append(s_ - cur_e)
            cur_s, cur_e = s_, e_
        else:
            cur_e = max(cur_e, e_)
    busy += cur_e - cur_s
    span = iv[-1][1] - iv[0][0]
    print(f"\nwall span {span / 1e6 / steps:.2f} ms/step, device busy (union) {busy / 1e6 / steps:.2f} "
          f"ms/step, idle {100 * (1 - busy / span):.1f} % in {len(gaps)} gaps "
          f"(largest {max(gaps or [0]) / 1e3:.1f} us); kernel-time sum / busy = {all_ms * 1e6 / busy:.2f}x "
          f"(stream concurrency)")


if __name__ == "__main__":
    main()
