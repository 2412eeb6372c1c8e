"""Writes tests/golden/stream_sha.json (run on an MI355X box): the sha256 of
the HOBE / FOBE record streams test_gpu_stream_pin.py pins."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.dirname(HERE)]
from test_gpu_stream_pin import stream_shas  # noqa: E402

if __name__ == "__main__":
  out = stream_shas()
  path = os.path.join(HERE, "stream_sha.json")
  with open(sys.argv[1] if len(sys.argv) > 1 else path, "w") as f:
    json.dump(out, f, indent=1, sort_keys=True)
  print(json.dumps(out))
