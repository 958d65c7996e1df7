"""Cityscapes reader -- drop-in for the reference's datasets/cityscapes.py:18-73.

File discovery (``**/*.png`` under the image and annotation roots, recursive), the id merge
(the first three ``_``-separated fields of the file name; ``*color.png`` annotations are the
colour maps, the others the train-id maps) and the (image, label) sample order are the
reference's.  Decoding is PIL (torchvision.io.read_image is not in this image): the image
comes out uint8 HWC [H, W, 3], the label uint8 [H, W].  Without transforms the sample is
returned raw; the device pipeline (rtsds_amd.transforms) turns batches of raw samples into
the network's NHWC input.  With reference-style callables in ``transform`` /
``target_transform`` they are applied to the raw tensors, as the reference does.
"""
import glob
import os
from collections import namedtuple

import numpy as np
import torch
from torch.utils.data import Dataset

class_names = [
    "road", "sidewalk", "building", "wall", "fence", "pole", "traffic light", "traffic sign",
    "vegetation", "terrain", "sky", "person", "rider", "car",
    "truck", "bus", "train", "motorcycle", "bicycle"
]


def read_png(path, rgb=False):
    """uint8 HWC (colour) / HW (grey) tensor of a PNG (the decode of torchvision.io.read_image;
    paletted label maps keep their palette indices, as read_image does)."""
    from PIL import Image
    with Image.open(path) as im:
        if rgb and im.mode != "RGB":
            im = im.convert("RGB")
        a = np.array(im)  # a writable copy (np.asarray of a PIL image is read-only)
    return torch.from_numpy(np.ascontiguousarray(a))


class CityScapes(Dataset):
    def __init__(self, annotation_path: str, images_path: str, transform=None, target_transform=None):
        super(CityScapes, self).__init__()
        images_path = self.__check_path__(images_path)
        annotation_path = self.__check_path__(annotation_path)
        self.images_filename = sorted(glob.glob(os.path.join(images_path, "**", "*.png"), recursive=True))
        self.annotations_filename = sorted(glob.glob(os.path.join(annotation_path, "**", "*.png"), recursive=True))
        self.image_dataset = self.__merge_ids__()
        self.transform = transform
        self.target_transform = target_transform

    def __check_path__(self, path: str) -> str:
        return path.rstrip("/\\")

    def __merge_ids__(self):
        def get_id(path: str) -> str:
            return "_".join(path.split("/")[-1].split("_")[:3])

        Image = namedtuple("Image", ["path", "labels"])
        img_set = {}
        for image in self.images_filename:
            img_set[get_id(image)] = Image(image, ["\0", "\0"])
        for label in self.annotations_filename:
            i = get_id(label)
            if i not in img_set:
                continue
            if label.endswith("color.png"):
                img_set[i].labels[1] = label
            else:
                img_set[i].labels[0] = label
        return list(img_set.values())

    def __getitem__(self, idx):
        if torch.is_tensor(idx):
            idx = idx.tolist()
        rec = self.image_dataset[idx]
        image = read_png(rec.path, rgb=True)
        label = read_png(rec.labels[0])
        if label.dim() == 3:  # an RGB-saved id map: the first channel holds the id
            label = label[..., 0].contiguous()
        if self.transform:
            image = self.transform(image)
        if self.target_transform:
            label = self.target_transform(label)
        return image, label

    def __len__(self):
        return len(self.image_dataset)
