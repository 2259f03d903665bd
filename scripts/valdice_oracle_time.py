"""How long one val-Dice oracle run takes on the box and where (diagnostics for sizing the seed-pair count):
fast host path per epoch, embeddings, oracle steps, evaluations. Uses oracle/ (test infrastructure)."""
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import valdice_protocol as P  # noqa: E402

cuda = torch.device("cuda", 0)
state, adam = P.load_warm()
runner = P.OracleRunner(cuda)
tr, va = P.SEEDS[0]
t = time.time()
b = P.fast_host_batches(tr, P.N_TRAIN, 0)
t_host0 = time.time() - t
t = time.time()
b = P.fast_host_batches(tr, P.N_TRAIN, 1)
t_host1 = time.time() - t
ref = runner.make(state, adam)
torch.cuda.synchronize()
t = time.time()
with P.oracle_mode():
    for i, x in enumerate(b):
        runner._embedding(ref, ("t", tr, i), x)
torch.cuda.synchronize()
t_emb = time.time() - t
t = time.time()
runner.train_steps(ref, tr, 1, limit=8)
torch.cuda.synchronize()
t_steps8 = time.time() - t
t = time.time()
c = runner.conf(ref, va)
t_conf = time.time() - t
t = time.time()
out, moved = runner.run(state, adam, tr, va)
t_run = time.time() - t
print(json.dumps({"host_epoch0_s": round(t_host0, 2), "host_epoch1_s": round(t_host1, 2),
                  "embed_16_batches_s": round(t_emb, 2), "steps8_s": round(t_steps8, 2), "conf_first_s": round(t_conf, 2),
                  "full_run_s": round(t_run, 2), "dice": [round(P.dice_of(c), 5) for _, c in out]}), flush=True)
