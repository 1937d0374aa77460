"""One VLP-16 scan through Pipeline.process_scan (diagnostics: run with LLSR_DEBUG_SYNC=1 to name a
faulting kernel)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "lego-loam-sr_amd"))
from llsr import Pipeline, default_config, synth  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 3
pipe = Pipeline(default_config("vlp16"), max_points=40000)
g = pipe.process_scan(synth.make_scan(seed, "vlp16"))
print("ok", g["n_segmented"], g["n_less_flat"])
