import os, sys, subprocess, json
sys.path.insert(0, 'tauv-vision_amd'); sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
from bench import build_model
model, oc, sd = build_model('fp16', torch.device('cuda', 0))
torch.manual_seed(0)
frames = torch.randint(0, 256, (1, 480, 640, 3), device='cuda', dtype=torch.uint8)
eng = model.engine(torch.device('cuda', 0), 480, 640)
out = eng.alloc_out(1)
eng.forward_u8(frames, out) if hasattr(eng, 'forward_u8') else None
torch.cuda.synchronize()
np.save(sys.argv[1], out.float().cpu().numpy())
ops = eng.profile(frames, out)
print(sum(1 for o in ops if o[3].endswith(', 1>') and 'c3::' in o[3]), 'SK launches')
