import os, sys, torch
sys.path.insert(0, os.environ["GRAFT_REPO_ROOT"])
import mmseg_amd
from bench import make_config
from mmseg_amd.data import device_batches
from mmseg_amd.models.build import build_model
from mmseg_amd.trainer.trainer import Trainer
dev = torch.device("cuda", 0)
cfg = make_config("dual_encoder", 2, "bf16")
torch.manual_seed(0)
tr = Trainer(cfg, build_model(cfg))
b = device_batches(2, 2, 96, 6, ["CT", "PET"], dev)
tr.train_step(b[0], 0)
prog = tr.model.backbone.__dict__["_engine"].program
for m in range(2):
    for l, blk in enumerate(prog.encs[m]):
        print("enc", m, l, blk.norm1_ok, blk.defer1, blk.defer_out)
for j, blk in enumerate(prog.dec.blocks):
    print("dec", j, blk.norm1_ok, blk.defer1, blk.defer_out)
