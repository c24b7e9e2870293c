"""3-D box container (reference: boxfusion/boxes.py:656-943, GeneralInstance3DBoxes).

xyz + lhw in `tensor` [N,6] and a full rotation `R` [N,3,3].  The geometry that the fusion path
runs every keyframe (`corners`, `transform2world`) executes in the gfx950 kernels
(bf_box_corners / bf_box_transform2world); tensors must live on the HIP device for those.
"""
from __future__ import annotations

import torch

from boxfusion_amd import _lib


class GeneralInstance3DBoxes:
    def __init__(self, xyzlhw, R, box_dim=15, origin=(0.5, 0.5, 0), dof=None):
        device = xyzlhw.device if isinstance(xyzlhw, torch.Tensor) else torch.device("cpu")
        self.tensor = torch.as_tensor(xyzlhw, dtype=torch.float32, device=device).clone()
        self.R = torch.as_tensor(R, dtype=torch.float32, device=device).clone()
        self.dof = dof
        self.box_dim = box_dim

    @classmethod
    def empty(cls, device="cpu"):
        return cls(torch.zeros((0, 6), device=device), torch.zeros((0, 3, 3), device=device))

    @property
    def device(self):
        return self.tensor.device

    @property
    def volume(self):
        return self.tensor[:, 3] * self.tensor[:, 4] * self.tensor[:, 5]

    @property
    def dims(self):
        return self.tensor[:, 3:6]

    @property
    def whl(self):
        return self.tensor[:, [5, 4, 3]]

    @property
    def xyzwhl(self):
        return self.tensor[:, [0, 1, 2, 5, 4, 3]]

    @property
    def gravity_center(self):
        return self.tensor[:, :3]

    center = gravity_center

    @property
    def corners(self):
        """[N,8,3] in the reference's v0..v7 order (boxes.py:725-778), on the GPU."""
        return _lib.box_corners(self.tensor, self.R)

    def transform2world(self, cam_pose):
        """xyz <- Rc xyz + tc, R <- Rc R in place (boxes.py:825-833)."""
        if not isinstance(cam_pose, torch.Tensor):
            cam_pose = torch.as_tensor(cam_pose)
        cam_pose = cam_pose.to(self.tensor.device, torch.float32).contiguous()
        self.tensor = self.tensor.contiguous()
        self.R = self.R.contiguous()
        _lib.box_transform2world(self.tensor, self.R, cam_pose)

    def translate(self, trans_vector):
        self.tensor[:, :3] += torch.as_tensor(trans_vector, device=self.tensor.device)

    @classmethod
    def _views(cls, tensor, R):
        """boxes over existing tensors, no copy (row slices of a larger box set)"""
        b = cls.__new__(cls)
        b.tensor, b.R, b.dof, b.box_dim = tensor, R, None, 15
        return b

    def __getitem__(self, item):
        if isinstance(item, int):
            return GeneralInstance3DBoxes(self.tensor[item].view(1, -1), self.R[item].view(1, 3, 3))
        if isinstance(item, slice) and (item.step is None or item.step == 1):
            return GeneralInstance3DBoxes._views(self.tensor[item], self.R[item])
        if isinstance(item, torch.Tensor) and item.dtype in (torch.int64, torch.int32) and item.dim() == 1:
            # a gather makes new tensors already: no second copy
            return GeneralInstance3DBoxes._views(self.tensor.index_select(0, item),
                                                 self.R.index_select(0, item))
        b, r = self.tensor[item], self.R[item]
        assert b.dim() == 2, f"Indexing on Boxes with {item} failed to return a matrix!"
        return GeneralInstance3DBoxes(b, r)

    def __len__(self):
        return self.tensor.shape[0]

    def __repr__(self):
        return f"GeneralInstance3DBoxes(\n    {self.tensor})"

    @classmethod
    def cat(cls, boxes_list):
        if len(boxes_list) == 0:
            return cls.empty()
        return cls._views(torch.cat([b.tensor for b in boxes_list], 0), torch.cat([b.R for b in boxes_list], 0))

    def split(self, sizes):
        return [GeneralInstance3DBoxes(t, r) for t, r in
                zip(torch.split(self.tensor, sizes), torch.split(self.R, sizes))]

    def to(self, device):
        return GeneralInstance3DBoxes(self.tensor.to(device), self.R.to(device))

    def clone(self):
        return GeneralInstance3DBoxes(self.tensor.clone(), self.R.clone())

    def __iter__(self):
        yield from self.tensor
