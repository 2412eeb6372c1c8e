"""Per-launch view of the dense-MLP engine from a rocprofv3 kernel trace:
the mlp_* kernels of each training batch in launch order (position in the
batch, not just the kernel name, so the two mlp_fwd<8> launches of the
combiner -- tower layer 1 and the head's hidden layer -- are told apart),
mean / median duration per position, and the mean gap before each launch.

  python tools/mlp_trace_summary.py <kernel_trace.csv> [--first-batch 200]
"""
import csv
import statistics
import sys


def main():
  path = sys.argv[1]
  skip = int(sys.argv[3]) if len(sys.argv) > 3 else 200
  rows = []
  for r in csv.DictReader(open(path)):
    n = r["Kernel_Name"]
    if "mlp_" not in n:
      continue
    short = n.replace("(anonymous namespace)::", "").replace("void ", "")
    short = short.split("((")[0].split("(")[0]
    rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short))
  rows.sort()
  # a batch starts at each mlp_fwd launch that follows a non-fwd launch
  batches, cur = [], []
  for s, e, n in rows:
    if n.startswith("mlp_fwd") and cur and not cur[-1][2].startswith("mlp_fwd"):
      batches.append(cur)
      cur = []
    cur.append((s, e, n))
  if cur:
    batches.append(cur)
  sig = {}
  for b in batches:
    sig.setdefault(tuple(x[2] for x in b), []).append(b)
  common = max(sig.items(), key=lambda kv: len(kv[1]))
  names, bs = common
  bs = bs[skip:] if len(bs) > 2 * skip else bs
  print("batches: %d (pattern of %d launches; %d other patterns)" %
        (len(bs), len(names), len(sig) - 1))
  tot = []
  for i, n in enumerate(names):
    d = [(b[i][1] - b[i][0]) / 1e3 for b in bs]
    g = [(b[i][0] - b[i - 1][1]) / 1e3 for b in bs] if i else [0.0]
    print("  %2d %-28s mean %7.2f  median %7.2f us   gap before %6.2f us" %
          (i, n, statistics.mean(d), statistics.median(d), statistics.mean(g)))
  span = [(b[-1][1] - b[0][0]) / 1e3 for b in bs]
  step = [(bs[k + 1][0][0] - bs[k][0][0]) / 1e3 for k in range(len(bs) - 1)] or [0]
  print("  batch span (first start -> last end) mean %.2f us; start-to-start "
        "median %.2f us" % (statistics.mean(span), statistics.median(step)))


if __name__ == "__main__":
  main()
