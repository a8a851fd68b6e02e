# eager vs eager bf16 C2 with lr=1e-4: gradient spread at step 1 (deterministic on/off)
import sys, torch
sys.path.insert(0, "/root/repo"); sys.path.insert(0, "/root/repo/tests")
import autoformer_amd as A, autoformer_amd.kernels as K
from autoformer_amd.detinit import det_init_, det_inputs
from autoformer_amd.train import TrainStep
from factory.AutoVC import AutoVC
A.set_compute("bf16")
for det in (False, True):
    K.set_deterministic(det)
    ms = []
    for _ in range(2):
        m = AutoVC(44, 256, 512, 16); det_init_(m); m = m.cuda().train(); ms.append((m, TrainStep(m, lr=1e-4)))
    bs = [tuple(torch.from_numpy(a).cuda() for a in det_inputs(64, 128, seed=40 + i)) for i in range(3)]
    for i, (x, e) in enumerate(bs):
        for m, t in ms: t.step(x, e)
        torch.cuda.synchronize()
        worst = max((((pa.grad - pb.grad).double().norm() / pa.grad.double().norm()).item(), n) for (n, pa), (_, pb) in zip(ms[0][0].named_parameters(), ms[1][0].named_parameters()))
        print(f"deterministic={det} step {i}: worst grad rel diff {worst[0]:.3e} {worst[1]}", flush=True)
    from autoformer_amd.layers import set_grad_sink
    set_grad_sink(False)
