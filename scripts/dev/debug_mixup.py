import sys, os
sys.path.insert(0, os.getcwd()); sys.path.insert(0, os.path.join(os.getcwd(), "tests"))
import numpy as np, torch
from test_sampling import _loader, _emulate
from golden_util import load
name = "sample_mixup_pad_n300"
loader, s = _loader(name, "cuda")
fx = load(name)
torch.manual_seed(s["seed"])
rows = loader._train_rows(0)
got = loader._gather([rows]).cpu().numpy()
emu = _emulate(loader.store.slab.cpu().numpy(), rows)
d = got != fx["bag"]
print("rows differing", np.unique(np.nonzero(d)[0]).size, "elements", d.sum(), "maxabs", np.abs(got - fx["bag"]).max())
print("emu==fixture", np.array_equal(emu, fx["bag"]), "got==emu", np.array_equal(got, emu))
r = np.unique(np.nonzero(d)[0])[:3]
i0 = rows.i0.numpy(); i1 = rows.i1.numpy()
for k in r:
    print(k, i0[k], i1[k], rows.wa[k].item(), rows.wb[k].item(), got[k, :4], fx["bag"][k, :4])
