"""KeyedJaggedTensor stand-in (golden generation only; see ../__init__.py)."""
import torch


class JaggedTensor:
    def __init__(self, values, lengths):
        self._values = values
        self._lengths = lengths

    def values(self):
        return self._values

    def lengths(self):
        return self._lengths

    def offsets(self):
        z = torch.zeros(1, dtype=torch.long, device=self._lengths.device)
        return torch.cat([z, torch.cumsum(self._lengths, 0)])


class KeyedJaggedTensor:
    def __init__(self, keys, values, lengths=None, offsets=None, **kw):
        self._keys = list(keys)
        self._values = values
        if lengths is None:
            lengths = offsets[1:] - offsets[:-1]
        self._lengths = lengths

    @staticmethod
    def from_lengths_sync(keys, values, lengths, **kw):
        return KeyedJaggedTensor(keys, values, lengths=lengths)

    def keys(self):
        return self._keys

    def values(self):
        return self._values

    def lengths(self):
        return self._lengths

    def to(self, device, non_blocking=False):
        return KeyedJaggedTensor(self._keys, self._values.to(device), self._lengths.to(device))

    def to_dict(self):
        stride = self._lengths.numel() // len(self._keys)
        out, pos = {}, 0
        for k_i, k in enumerate(self._keys):
            ln = self._lengths[k_i * stride:(k_i + 1) * stride]
            n = int(ln.sum())
            out[k] = JaggedTensor(self._values[pos:pos + n], ln)
            pos += n
        return out
