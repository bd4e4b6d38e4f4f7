"""Drop-in for dl_code/pcode/utils/tensor_buffer.py (flat buffer + per-tensor views).

Difference from the reference: the flat buffer keeps the dtype of the packed
tensors (the reference's `flatten` always allocates the default float dtype,
communication.py:69-72, which silently turns int64 indices into fp32).
"""
import torch


def flatten(tensors, shapes=None, use_cuda=True):
    pointers = [0]
    if shapes is not None:
        for shape in shapes:
            pointers.append(pointers[-1] + shape[1])
    else:
        for tensor in tensors:
            pointers.append(pointers[-1] + tensor.nelement())
    dev = tensors[0].device if (tensors[0].is_cuda and use_cuda) else "cpu"
    vec = torch.empty(pointers[-1], dtype=tensors[0].dtype, device=dev)
    for tensor, start, end in zip(tensors, pointers[:-1], pointers[1:]):
        vec[start:end] = tensor.data.view(-1)
    return vec


class TensorBuffer:
    def __init__(self, tensors, use_cuda=True):
        indices = [0]
        for tensor in tensors:
            indices.append(indices[-1] + tensor.nelement())
        self._start_idx = indices[:-1]
        self._end_idx = indices[1:]
        self._tensors_len = len(tensors)
        self._tensors_sizes = [x.size() for x in tensors]
        self.buffer = flatten(tensors, use_cuda=use_cuda)  # copies

    @classmethod
    def from_flat(cls, buffer, sizes):
        """Wrap an existing flat buffer (no copy) with per-tensor sizes."""
        self = cls.__new__(cls)
        indices = [0]
        for s in sizes:
            n = 1
            for d in s:
                n *= d
            indices.append(indices[-1] + n)
        self._start_idx = indices[:-1]
        self._end_idx = indices[1:]
        self._tensors_len = len(sizes)
        self._tensors_sizes = [torch.Size(s) for s in sizes]
        self.buffer = buffer
        return self

    def __getitem__(self, index):
        return self.buffer[self._start_idx[index]:self._end_idx[index]].view(self._tensors_sizes[index])

    def __len__(self):
        return self._tensors_len

    def is_cuda(self):
        return self.buffer.is_cuda

    def nelement(self):
        return self.buffer.nelement()

    def unpack(self, tensors):
        for tensor, entry in zip(tensors, self):
            tensor.data[:] = entry
