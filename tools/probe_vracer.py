"""GPU probe: create VRACER handles of growing size and run one forward."""
import sys
import numpy as np
from korali_amd.vracer import VracerDevice

for E in (64, 4096):
    d = VracerDevice(environments=E, hidden_size=64, hidden_layers=1, mini_batch_size=64, replay_maximum_size=1024,
                     replay_start_size=512)
    print("create ok", E, d.hyperparameter_count, flush=True)
    out = d.run_policy(np.zeros((8, 4), np.float32))
    print("policy ok", out[0], flush=True)
    d.close()
print("done")
