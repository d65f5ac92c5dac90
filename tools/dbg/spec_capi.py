"""debug: the torch-free composite build with the speculative FFTs on / off, per-q W_q diff"""
import os, subprocess, sys
import numpy as np
HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
W = os.path.join(ROOT, "tests", "capi_worker.py")
case = sys.argv[1] if len(sys.argv) > 1 else "toy222"
outs = {}
for tag, env in [("s0", {"FISDF_FIT_SPEC": "0"}), ("s1", {"FISDF_FIT_SPEC": "1"}),
                 ("s1sync", {"FISDF_FIT_SPEC": "1", "FISDF_DBG_SPEC_SYNC": "1"}),
                 ("s1again", {"FISDF_FIT_SPEC": "1"})]:
    out = f"/tmp/spec_{tag}.npz"
    e = dict(os.environ, **env)
    p = subprocess.run([sys.executable, W, case, out], env=e, timeout=200)
    if p.returncode:
        print(tag, "worker failed", p.returncode); sys.exit(1)
    outs[tag] = dict(np.load(out))
a = outs["s0"]
print("ranks", a["ranks"], "min_norm", a["min_norm"], "nfit", a["nfit"])
for tag, o in outs.items():
    d = [float(abs(o["wq"][q] - a["wq"][q]).max()) for q in range(a["wq"].shape[0])]
    print(tag, "ranks", o["ranks"], "perm same", np.array_equal(o["perm"], a["perm"]),
          "dvj %.2e dvk %.2e" % (abs(o["vj"] - a["vj"]).max(), abs(o["vk"] - a["vk"]).max()),
          "per-q dW", ["%.1e" % x for x in d], flush=True)
