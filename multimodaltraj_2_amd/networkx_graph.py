"""Online pedestrian graph of the reference (networkx_graph.py), host side.

The reference keeps one networkx MultiDiGraph node per pedestrian with a
``node_pos_list`` [8, 2] slot array and reads it back with
``get_node_attr('node_pos_list')`` (networkx_graph.py:30-73, 114-150).  Only
that tensor content reaches the hot path, so this mirror stores the nodes in
an insertion-ordered dict (no networkx, no per-node torch state tensors:
networkx_graph.py:167-168 allocates them but nothing reads them) and keeps the
same update rules:

* a node seen for the first time is created with ``node_pos_list = zeros``
  (its position is NOT written, networkx_graph.py:123-129);
* a node seen again gets ``node_pos_list[itr] = pos`` where ``itr`` is the
  frame's ordinal in the batch; ``itr >= 8`` is dropped (IndexError, :117-120);
* a pedestrian without targets is skipped (KeyError, :60-68);
* the graph is never reset between batches (quirk Q19).

``scene_tensors`` turns a batch into the [W, N, 2] position window the HIP
step consumes, for the train.py node slice (quirk Q10) or the sample.py time
slice.
"""
from __future__ import annotations

import numpy as np

POS_LIST_LEN = 8     # networkx_graph.py:114 pos_list_len


class Graph:
    """Insertion-ordered node store with the reference's attribute names."""

    def __init__(self):
        self.nodes = {}          # node id -> attribute dict
        self.dist_mat = np.zeros((1, 1))
        self.step = 0

    def getNodes(self):
        return self.nodes

    def setNodes(self, framenum, node_id, pos, targets):
        """``targets``: the node's target list attribute (Node.targets)."""
        rec = self.nodes.get(node_id)
        if rec is None:
            self.nodes[node_id] = {"seq": [], "node_pos_list": np.zeros((POS_LIST_LEN, 2)),
                                   "targets": targets, "vel": 0}
        elif 0 <= framenum < POS_LIST_LEN:
            rec["node_pos_list"][framenum] = pos

    def get_node_attr(self, param):
        return {k: v[param] for k, v in self.nodes.items()}

    def delGraph(self, framenum=None):
        self.nodes.clear()


class online_graph:
    def __init__(self, args):
        self.diff = args.seq_length
        self.batch_size = args.batch_size
        self.onlineGraph = Graph()

    def reset_graph(self, framenum=None):
        self.onlineGraph.delGraph(framenum)

    def ConstructGraph(self, current_batch, future_traj, framenum, stateful=True, valid=False):
        """networkx_graph.py:30-73 semantics (float framenum cast to int, Q9)."""
        framenum = int(framenum)
        g = self.onlineGraph
        g.step = framenum
        if valid:
            for ped, pos in current_batch.items():
                tg = [future_traj[ped]] if (framenum > 0 and framenum % 8) else []
                g.setNodes(framenum, ped, [pos], tg)
            return g
        for itr, key in enumerate(current_batch):
            for entry in current_batch[key]:
                (ped, pos), = entry.items()
                ped = int(ped)
                if ped not in future_traj:
                    continue
                seq = future_traj[ped]
                if len(seq) < framenum:
                    tg = seq[0:12]
                elif len(seq[framenum:framenum + 12]) < 12:
                    tg = seq
                else:
                    tg = seq[framenum:framenum + 12]
                g.setNodes(itr, ped, pos, [tg])
        return g


def batch_v(node_pos_list, obs_len=8, frame=1, mode="train"):
    """Bv of train.py:76-85 (``mode='train'``: the node slice
    [frame:frame+obs_len], quirk Q10) or sample.py:152-164 (``mode='sample'``:
    the time slice).  Returns [obs_len, N]."""
    npl = np.asarray(node_pos_list, dtype=np.float64).reshape(-1, POS_LIST_LEN, 2)
    if mode == "train":
        sl = npl[frame:frame + obs_len]
        bv = np.linalg.norm(sl, axis=2).reshape(len(sl), POS_LIST_LEN)
        return np.transpose(bv)
    return np.transpose(np.linalg.norm(npl[:, 0:obs_len], axis=2))


def scene_tensors(node_pos_list, obs_len=8, frame=1, mode="train"):
    """Position window [obs_len, N, 2] such that the HIP step's window norms
    equal ``batch_v(..)``: train mode window[t, i] = node_pos_list[frame+i][t],
    sample mode window[t, i] = node_pos_list[i][t]."""
    npl = np.asarray(node_pos_list, dtype=np.float64).reshape(-1, POS_LIST_LEN, 2)
    if mode == "train":
        sl = npl[frame:frame + obs_len]                  # [N, 8, 2]
        return np.ascontiguousarray(np.transpose(sl, (1, 0, 2))[:obs_len])
    return np.ascontiguousarray(np.transpose(npl[:, 0:obs_len], (1, 0, 2)))
