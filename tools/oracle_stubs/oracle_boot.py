"""Import-time shims for running the unmodified reference in this container
(fixture generation only). Inserts a no-op tensorboard SummaryWriter."""
import sys
import types

_tb = types.ModuleType("torch.utils.tensorboard")


class SummaryWriter:  # noqa: D401
    def __init__(self, *a, **k):
        pass

    def add_text(self, *a, **k):
        pass

    def add_scalar(self, *a, **k):
        pass

    def close(self):
        pass


_tb.SummaryWriter = SummaryWriter
sys.modules["torch.utils.tensorboard"] = _tb
