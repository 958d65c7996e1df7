"""GTA5 reader -- drop-in for the reference's datasets/gta5.py:50-118.

Images and labels are matched by file stem (``images/*.png`` / ``labels/*.png``); the label is
the stored id map, or -- with ``in_getting_decoder=True`` -- the RGB colour map decoded to train
ids (gta5.py:111-118: a pixel gets id i when its colour is train id i's Cityscapes colour,
else 0), on the device by rtsds_gta5_decode when the label is decoded by
rtsds_amd.transforms.decode_gta5_labels.  Samples are uint8 HWC as in datasets/cityscapes.py.
"""
import glob
import os
from collections import namedtuple

import torch
from torch.utils.data import Dataset

from .cityscapes import read_png

# train id -> Cityscapes colour (the ids 0..18 of gta5.py:10-44's colour map)
TRAIN_ID_COLORS = [
    (128, 64, 128), (244, 35, 232), (70, 70, 70), (102, 102, 156), (190, 153, 153), (153, 153, 153),
    (250, 170, 30), (220, 220, 0), (107, 142, 35), (152, 251, 152), (70, 130, 180), (220, 20, 60),
    (255, 0, 0), (0, 0, 142), (0, 0, 70), (0, 60, 100), (0, 80, 100), (0, 0, 230), (119, 11, 32)]


class GTA5(Dataset):
    def __init__(self, images_path, labels_path, transformer, target_transofrmer, in_getting_decoder=False):
        super(GTA5, self).__init__()
        self.transform = transformer
        self.target_transform = target_transofrmer
        self.in_getting_decoder = in_getting_decoder
        self.images_filenames = sorted(glob.glob(os.path.join(images_path, "**.png")))
        self.labels_filenames = sorted(glob.glob(os.path.join(labels_path, "**.png")))
        self.images_dataset = self.__make_dataset__()

    def label_driver(self, label_path: str):
        """RGB label -> train ids [1, H, W] int64 (gta5.py:64-67), on the device."""
        from ..transforms import decode_gta5_labels
        rgb = read_png(label_path, rgb=True)
        return decode_gta5_labels(rgb.cuda()).unsqueeze(0)

    def __getitem__(self, idx):
        if torch.is_tensor(idx):
            idx = idx.tolist()
        rec = self.images_dataset[idx]
        image = read_png(rec.image, rgb=True)
        if self.in_getting_decoder:
            label = read_png(rec.label[0], rgb=True)  # decoded on the device after batching
        else:
            label = read_png(rec.label[0])
            if label.dim() == 3:
                label = label[..., 0].contiguous()
        if self.transform:
            image = self.transform(image)
        if self.target_transform:
            label = self.target_transform(label)
        return image, label

    def __make_dataset__(self):
        def get_id(path):
            return os.path.splitext(os.path.basename(path))[0]

        Image = namedtuple("Image", ["image", "label"])
        img_set = {}
        for image in self.images_filenames:
            img_set[get_id(image)] = Image(image, ["\0"])
        for label in self.labels_filenames:
            i = get_id(label)
            if i in img_set:
                img_set[i].label[0] = label
        return list(img_set.values())

    def __len__(self):
        return len(self.images_filenames)
