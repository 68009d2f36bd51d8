#!/usr/bin/env python3
"""Timeline of the last forward in a rocprofv3 kernel trace: every kernel of the last LSTM launch's
window, start / end relative to the LSTM start (us), grouped by kernel class.

    python tools/trace_timeline.py gpurun_out/prof_x/run_kernel_trace.csv [pick]

pick: which LSTM launch (python index, default -3: bench.py ends with a per-class timing pass and an
isolated pass of the dominant class after the timed forwards)
"""
import csv
import sys


def short(n):
    for k in ("lstm_pair", "lstm_resident", "conv01", "convk4", "gemm2_kernelIDF16b", "gemm2_kernel<float", "attn4", "attn3", "block_kernel", "block3", "heads_kernel",
              "lnproj_kernel", "rowpanel", "streamOpsWait", "streamOpsWrite", "probs", "labels", "vad_head",
              "zero_rows", "copyBuffer", "layernorm"):
        if k in n:
            return k
    return n[:40]


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows]
    ks.sort()
    lstm = [k for k in ks if k[2] in ("lstm_resident", "lstm_pair")]
    pick = int(sys.argv[2]) if len(sys.argv) > 2 else -3
    L = lstm[pick] if len(lstm) >= -pick else lstm[0]  # the last timed forward
    t0 = L[0]
    win = [k for k in ks if k[0] >= L[0] - 3_000_000 and k[0] <= L[1] + 3_000_000]
    prev_end = None
    print(f"LSTM {L[0]-t0} .. {(L[1]-t0)/1e3:.1f} us (queue {L[3]})")
    for s, e, n, q in win:
        if n in ("lstm_resident", "lstm_pair"):
            continue
        gap = "" if prev_end is None else f" gap {(s - prev_end)/1e3:7.1f}"
        print(f"{(s - t0)/1e3:9.1f} {(e - t0)/1e3:9.1f} {(e - s)/1e3:8.1f} q{q} {n}{gap}")
        prev_end = e


if __name__ == "__main__":
    main()
