"""Elastic training scenarios (launched by tests/test_elastic_cpu.py through mihvdrun --min-np).

usage: python elastic_worker.py <scenario> <outdir>
  shrink : 3 workers; worker 2 dies at step 9 (first life) -> the survivors roll back to the last
           commit and finish with 2 workers.
  respawn: same failure with --respawn: a replacement worker joins and receives the state.
  grow   : 2 workers; rank 0 asks the launcher for one more worker (SIGUSR1) at step 6 -> commit()
           raises HostsUpdatedInterrupt everywhere, the world re-forms with 3 workers.
"""
import json
import os
import signal
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import mihvd.torch as hvd  # noqa: E402

STEPS = 24


def main():
    scenario, outdir = sys.argv[1], sys.argv[2]
    wid = int(os.environ["MIHVD_WORKER_ID"])
    hvd.init()
    torch.manual_seed(0)
    model = torch.nn.Sequential(torch.nn.Linear(8, 16), torch.nn.Tanh(), torch.nn.Linear(16, 2))
    opt = hvd.DistributedOptimizer(torch.optim.SGD(model.parameters(), lr=0.05),
                                   named_parameters=model.named_parameters())
    state = hvd.elastic.TorchState(model, opt, step=0, sizes=[], resets=0)

    def on_reset():
        state.resets += 1

    state.register_reset_callbacks([on_reset])

    @hvd.elastic.run
    def train(state):
        while state.step < STEPS:
            if scenario in ("shrink", "respawn") and wid == 2 and state.step == 9:
                os._exit(3)  # a worker dies mid-training (after its step-8 commit)
            if scenario == "grow" and hvd.rank() == 0 and state.step == 6 and hvd.size() == 2:
                os.kill(os.getppid(), signal.SIGUSR1)
                time.sleep(1.0)  # let the launcher publish the new generation
            g = torch.Generator().manual_seed(1000 * state.step + hvd.rank())
            x = torch.randn(16, 8, generator=g)
            y = torch.randn(16, 2, generator=g)
            opt.zero_grad()
            torch.nn.functional.mse_loss(model(x), y).backward()
            opt.step()
            state.step += 1
            state.sizes.append(hvd.size())
            if state.step % 2 == 0:
                state.commit()

    train(state)
    params = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    sig = [float(v) for v in hvd.allgather(params[:8].reshape(1, -1)).reshape(-1)]
    with open(os.path.join(outdir, f"{scenario}.w{wid}.json"), "w") as f:
        json.dump({"wid": wid, "rank": hvd.rank(), "size": hvd.size(), "step": state.step, "sizes": state.sizes,
                   "resets": state.resets, "allgathered": sig}, f)
    hvd.shutdown()


if __name__ == "__main__":
    main()
