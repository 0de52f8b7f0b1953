"""Client-value plumbing shared by the aggregators.

TFF hands an aggregation process a list of client tensors at CLIENTS and
expects the result at SERVER.  Here client values may be numpy arrays / lists
(host, as the TFF simulation executor holds them: copied H2D once) or torch
device tensors (already resident: no copy), either as a list or stacked
[C, *shape].  Results come back on the host when the inputs were host values.
"""
import numpy as np
import torch


def to_device_rows(client_values, dtype=torch.float32):
  """Returns (rows: list of contiguous 1-D cuda tensors, shape, host_input)."""
  if isinstance(client_values, torch.Tensor):
    host = not client_values.is_cuda
    t = client_values.to(device="cuda", dtype=dtype)
    shape = tuple(t.shape[1:])
    flat = t.reshape(t.shape[0], -1).contiguous()
    return [flat[i] for i in range(flat.shape[0])], shape, host
  rows, shape, host = [], None, False
  for v in client_values:
    if isinstance(v, torch.Tensor):
      host = host or not v.is_cuda
      t = v.to(device="cuda", dtype=dtype)
    else:
      host = True
      t = torch.from_numpy(np.ascontiguousarray(np.asarray(v, dtype=torch_to_np(dtype)))).cuda()
    if shape is None:
      shape = tuple(t.shape)
    elif tuple(t.shape) != shape:
      raise ValueError("client values must share one shape, got %s and %s" % (shape, tuple(t.shape)))
    rows.append(t.reshape(-1).contiguous())
  if not rows:
    raise ValueError("no client values")
  return rows, shape, host


def torch_to_np(dtype):
  return {torch.float32: np.float32, torch.int32: np.int32}[dtype]


def finish(t, shape, host):
  t = t.reshape(shape)
  return t.cpu().numpy() if host else t


def sharded_rows(value, shape, sharded, multi, group=None):
  """Client rows of one rank's block for a sharded round.

  Returns (rows, host, lo, base): ``lo`` is this rank's first global client index
  and ``base`` one clock base for the whole round (distributed.round_preamble),
  both None unless ``multi``.  Under ``multi`` a rank whose values are rejected
  (shape) still joins the preamble's all-reduce, and then EVERY rank raises -- a
  rank raising alone would leave the others blocked in the round's collectives.
  """
  from federated_amd import distributed  # pylint: disable=g-import-not-at-top
  rows, host, bad = [], False, None
  if not (sharded and len(value) == 0):
    try:
      rows, vshape, host = to_device_rows(value, torch.float32)
      if vshape != tuple(shape):
        raise ValueError("client value shape %s != %s" % (vshape, tuple(shape)))
    except Exception as e:  # pylint: disable=broad-except
      # any rejection (ValueError for a shape, TypeError / RuntimeError for a dtype or
      # device) is flagged through the preamble, so no rank raises alone
      if not multi:
        raise
      bad = e
  if not multi:
    return rows, host, None, None
  lo, _, any_bad, base = distributed.round_preamble(len(rows), bad is not None, group)
  if any_bad:
    raise bad if bad is not None else ValueError("client values rejected on another rank")
  return rows, host, lo, base
