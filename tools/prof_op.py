import cProfile, pstats, sys, os, io
sys.path.insert(0, os.environ.get("GRAFT_REPO_ROOT", "."))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "."), "tools"))
import torch
import opbench
dev = torch.device("cuda:0")
opbench.run(16, 16, 16, 50, dev, True)
pr = cProfile.Profile()
pr.enable()
opbench.run(16, 16, 16, 300, dev, True)
pr.disable()
s = io.StringIO()
pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(30)
print(s.getvalue()[:6000])
