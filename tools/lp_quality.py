"""LP_NODE_EDGE_CLASSIFIER accuracy of FOBE embeddings trained on the GPU vs
by the CPU oracle on the reference's snap_youtube_tiny fixture, over seeds
(the end-to-end quality signal of SURVEY §8f rank 3). JSON to argv[1]."""
import json, os, random, sys, time
import numpy as np
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]
from hypergraphembedding_amd import EmbedHg2vBoolean, EmbedHg2vAlgDist, Hypergraph
from hypergraphembedding_amd.evaluation_util import (
    LinkPredictionData, RemoveRandomConnections, RunLinkPredictionExperiment,
    SampleMissingConnections)
from test_gpu_lp_combine import _oracle_fobe_embedding

hg = Hypergraph()
with open(os.path.join(ROOT, "tests", "golden", "snap_youtube_tiny.hypergraph.pb"), "rb") as f:
  hg.ParseFromString(f.read())
out = {"graph": "snap_youtube_tiny (reference fixture)", "removal_prob": 0.1,
       "dim": 16, "runs": []}
for seed in range(int(sys.argv[2]) if len(sys.argv) > 2 else 4):
  random.seed(seed); np.random.seed(seed)
  sub, removed = RemoveRandomConnections(hg, 0.1)
  bad = SampleMissingConnections(hg, len(removed))
  run = {"seed": seed, "removed": len(removed)}
  embs = {}
  t = time.time(); embs["gpu_fobe"] = EmbedHg2vBoolean(sub, 16); run["gpu_fobe_s"] = round(time.time() - t, 2)
  t = time.time(); embs["cpu_oracle_fobe"] = _oracle_fobe_embedding(sub, 16, seed); run["cpu_oracle_fobe_s"] = round(time.time() - t, 2)
  embs["gpu_hobe"] = EmbedHg2vAlgDist(sub, 16)
  for name, emb in embs.items():
    np.random.seed(100 + seed); random.seed(100 + seed)
    m = RunLinkPredictionExperiment(LinkPredictionData(sub, emb, removed, bad, 0.1),
                                    "LP_NODE_EDGE_CLASSIFIER")
    run[name] = {"accuracy": round(m.accuracy, 4), "f1": round(m.f1, 4)}
  print(json.dumps(run), flush=True)
  out["runs"].append(run)
for k in ("gpu_fobe", "cpu_oracle_fobe", "gpu_hobe"):
  out[k + "_mean_accuracy"] = round(float(np.mean([r[k]["accuracy"] for r in out["runs"]])), 4)
json.dump(out, open(sys.argv[1], "w"), indent=1)
print(json.dumps({k: v for k, v in out.items() if k != "runs"}))
