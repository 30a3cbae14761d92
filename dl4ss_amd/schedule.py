"""Learning-rate schedules of the reference drivers.

* ``TDAA_beta/main_run_sstune_EvalVer.py:570-575``: at the start of every epoch with
  ``epoch_idx % 10 == 0`` each param group's lr is halved while it is ``>= 1e-7`` (so the
  first halving happens at epoch 0: training runs at 1e-4 from the start).
* ``Torch_multi/main_run_multi_selfSS_dB.py:441-444``: halved every 50 epochs, no floor.
* ``main_run_sstune_cRM_EvalVer.py:627-631`` has the 50-epoch / ``>= 5e-6`` form switched
  off (``if 0 and ...``): a constant lr.

``SepTrainer.lr`` is read by every Adam launch, so applying a schedule is assigning it.
"""


class LRHalving:
    def __init__(self, lr, every, floor=None, enabled=True):
        self.lr, self.every, self.floor, self.enabled = lr, every, floor, enabled

    def at_epoch_start(self, epoch_idx):
        """The reference's per-epoch update; returns the lr for this epoch."""
        if self.enabled and epoch_idx % self.every == 0:
            if self.floor is None or self.lr >= self.floor:
                self.lr /= 2
        return self.lr

    def apply(self, trainer, epoch_idx):
        trainer.lr = self.at_epoch_start(epoch_idx)
        return trainer.lr


def evalver(lr=2e-4):
    """EvalVer.py:570-575."""
    return LRHalving(lr, every=10, floor=1e-7)


def selfss_db(lr=2e-4):
    """selfSS_dB.py:442-444."""
    return LRHalving(lr, every=50, floor=None)


def crm_evalver(lr=2e-4):
    """cRM_EvalVer.py:627 (disabled in the reference)."""
    return LRHalving(lr, every=50, floor=5e-6, enabled=False)
