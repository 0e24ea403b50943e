"""Find where a training step's copies and fills come from (torch.profiler on the GPU).

    python tools/copy_probe.py

Prints aten copy_/fill_/zero_ counts by input shape and, for every 4-D copy,
the chain of parent ops (autograd backward nodes included).  Used for
profiles/README.md finding 13.
"""
import sys, os
sys.path.insert(0, os.getcwd())
import torch
from torch.profiler import profile, ProfilerActivity
from distributed_model_parallel_amd.train.step import StepConfig, build_train_state
from distributed_model_parallel_amd.utils.env import init_distributed, destroy_distributed
env = init_distributed()
cfg = StepConfig(model="resnet50", batch_size=32, image_size=224, dtype=torch.bfloat16, parallel="ddp")
st = build_train_state(cfg, env.device)
for _ in range(3): st.step()
torch.cuda.synchronize()
with profile(activities=[ProfilerActivity.CPU], record_shapes=True, with_stack=True) as prof:
    st.step(); torch.cuda.synchronize()
ka = prof.key_averages(group_by_input_shape=True)
for e in ka:
    if e.key in ("aten::copy_", "aten::fill_", "aten::zero_", "aten::zeros", "aten::add_", "aten::add"):
        print("==", e.key, e.count, str(e.input_shapes)[:300])
evs = prof.events()
for i, e in enumerate(evs):
    if e.name == "aten::copy_" and e.input_shapes and len(e.input_shapes[0]) == 4:
        par = e.cpu_parent
        chain = []
        while par is not None and len(chain) < 6:
            chain.append(par.name); par = par.cpu_parent
        print("COPY", e.input_shapes, " <- ".join(chain))
destroy_distributed()
