"""Training-time augmentation (reference `core/utils/augmentor.py`).

``FlowAugmentor`` (dense GT: Chairs / Things / Sintel) and ``SparseFlowAugmentor`` (KITTI / HD1K)
reproduce the reference pipelines step for step -- photometric jitter (asymmetric with p=0.2 for the
dense one), eraser occlusion (p=0.5, 1-2 boxes of mean colour), random scale 2^U(min,max) with
stretch, flips, random crop (sparse: with margins) -- and the same probabilities and ranges.

OpenCV / torchvision are not used: resizing is the native OpenCV-compatible bilinear resize
(``utils.imgproc.resize_linear``) and ``ColorJitter`` is re-implemented on PIL's ImageEnhance / HSV
exactly as torchvision does for PIL images (factors from the same ranges, random order of the four
ops drawn with ``torch.randperm``).
"""
import numpy as np
import torch
from PIL import Image, ImageEnhance

from ..utils.imgproc import resize_linear


class ColorJitter:
    """torchvision.transforms.ColorJitter for PIL images (brightness, contrast, saturation, hue)."""

    def __init__(self, brightness=0.0, contrast=0.0, saturation=0.0, hue=0.0):
        self.brightness = self._range(brightness)
        self.contrast = self._range(contrast)
        self.saturation = self._range(saturation)
        self.hue = None if hue == 0 else (-hue, hue)

    @staticmethod
    def _range(v):
        return None if v == 0 else (max(0.0, 1.0 - v), 1.0 + v)

    @staticmethod
    def _uniform(lo, hi):
        return float(torch.empty(1).uniform_(lo, hi))

    @staticmethod
    def adjust_hue(img, factor):
        if abs(factor) < 1e-12:
            return img
        mode = img.mode
        h, s, v = img.convert('HSV').split()
        nh = np.array(h, dtype=np.uint8)
        with np.errstate(over='ignore'):
            nh = (nh.astype(np.int16) + int(np.round(factor * 255))) % 256
        h = Image.fromarray(nh.astype(np.uint8), 'L')
        return Image.merge('HSV', (h, s, v)).convert(mode)

    def __call__(self, img):
        order = torch.randperm(4).tolist()
        b = None if self.brightness is None else self._uniform(*self.brightness)
        c = None if self.contrast is None else self._uniform(*self.contrast)
        s = None if self.saturation is None else self._uniform(*self.saturation)
        h = None if self.hue is None else self._uniform(*self.hue)
        for fn in order:
            if fn == 0 and b is not None:
                img = ImageEnhance.Brightness(img).enhance(b)
            elif fn == 1 and c is not None:
                img = ImageEnhance.Contrast(img).enhance(c)
            elif fn == 2 and s is not None:
                img = ImageEnhance.Color(img).enhance(s)
            elif fn == 3 and h is not None:
                img = self.adjust_hue(img, h)
        return img


def _eraser(img1, img2, prob, lo=50, hi=100):
    ht, wd = img1.shape[:2]
    if np.random.rand() < prob:
        mean_color = np.mean(img2.reshape(-1, 3), axis=0)
        for _ in range(np.random.randint(1, 3)):
            x0 = np.random.randint(0, wd)
            y0 = np.random.randint(0, ht)
            dx = np.random.randint(lo, hi)
            dy = np.random.randint(lo, hi)
            img2[y0:y0 + dy, x0:x0 + dx, :] = mean_color
    return img1, img2


class FlowAugmentor:
    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=True):
        self.crop_size = crop_size
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.spatial_aug_prob = 0.8
        self.stretch_prob = 0.8
        self.max_stretch = 0.2
        self.do_flip = do_flip
        self.h_flip_prob = 0.5
        self.v_flip_prob = 0.1
        self.photo_aug = ColorJitter(brightness=0.4, contrast=0.4, saturation=0.4, hue=0.5 / 3.14)
        self.asymmetric_color_aug_prob = 0.2
        self.eraser_aug_prob = 0.5

    def color_transform(self, img1, img2):
        if np.random.rand() < self.asymmetric_color_aug_prob:
            img1 = np.array(self.photo_aug(Image.fromarray(img1)), dtype=np.uint8)
            img2 = np.array(self.photo_aug(Image.fromarray(img2)), dtype=np.uint8)
        else:
            stack = np.concatenate([img1, img2], axis=0)
            stack = np.array(self.photo_aug(Image.fromarray(stack)), dtype=np.uint8)
            img1, img2 = np.split(stack, 2, axis=0)
        return img1, img2

    def eraser_transform(self, img1, img2, bounds=(50, 100)):
        return _eraser(img1, img2, self.eraser_aug_prob, bounds[0], bounds[1])

    def spatial_transform(self, img1, img2, flow):
        ht, wd = img1.shape[:2]
        min_scale = np.maximum((self.crop_size[0] + 8) / float(ht), (self.crop_size[1] + 8) / float(wd))
        scale = 2 ** np.random.uniform(self.min_scale, self.max_scale)
        scale_x = scale_y = scale
        if np.random.rand() < self.stretch_prob:
            scale_x *= 2 ** np.random.uniform(-self.max_stretch, self.max_stretch)
            scale_y *= 2 ** np.random.uniform(-self.max_stretch, self.max_stretch)
        scale_x = np.clip(scale_x, min_scale, None)
        scale_y = np.clip(scale_y, min_scale, None)
        if np.random.rand() < self.spatial_aug_prob:
            img1 = resize_linear(img1, fx=scale_x, fy=scale_y)
            img2 = resize_linear(img2, fx=scale_x, fy=scale_y)
            flow = resize_linear(flow, fx=scale_x, fy=scale_y)
            flow = flow * [scale_x, scale_y]
        if self.do_flip:
            if np.random.rand() < self.h_flip_prob:
                img1, img2 = img1[:, ::-1], img2[:, ::-1]
                flow = flow[:, ::-1] * [-1.0, 1.0]
            if np.random.rand() < self.v_flip_prob:
                img1, img2 = img1[::-1, :], img2[::-1, :]
                flow = flow[::-1, :] * [1.0, -1.0]
        y0 = np.random.randint(0, img1.shape[0] - self.crop_size[0])
        x0 = np.random.randint(0, img1.shape[1] - self.crop_size[1])
        sl = (slice(y0, y0 + self.crop_size[0]), slice(x0, x0 + self.crop_size[1]))
        return img1[sl], img2[sl], flow[sl]

    def __call__(self, img1, img2, flow):
        img1, img2 = self.color_transform(img1, img2)
        img1, img2 = self.eraser_transform(img1, img2)
        img1, img2, flow = self.spatial_transform(img1, img2, flow)
        return (np.ascontiguousarray(img1), np.ascontiguousarray(img2),
                np.ascontiguousarray(flow, dtype=np.float32))


class SparseFlowAugmentor:
    def __init__(self, crop_size, min_scale=-0.2, max_scale=0.5, do_flip=False):
        self.crop_size = crop_size
        self.min_scale = min_scale
        self.max_scale = max_scale
        self.spatial_aug_prob = 0.8
        self.stretch_prob = 0.8
        self.max_stretch = 0.2
        self.do_flip = do_flip
        self.h_flip_prob = 0.5
        self.v_flip_prob = 0.1
        self.photo_aug = ColorJitter(brightness=0.3, contrast=0.3, saturation=0.3, hue=0.3 / 3.14)
        self.asymmetric_color_aug_prob = 0.2
        self.eraser_aug_prob = 0.5

    def color_transform(self, img1, img2):
        stack = np.concatenate([img1, img2], axis=0)
        stack = np.array(self.photo_aug(Image.fromarray(stack)), dtype=np.uint8)
        return tuple(np.split(stack, 2, axis=0))

    def eraser_transform(self, img1, img2):
        return _eraser(img1, img2, self.eraser_aug_prob)

    def resize_sparse_flow_map(self, flow, valid, fx=1.0, fy=1.0):
        """Scatter the valid sparse samples into the resized grid (no interpolation across holes)."""
        ht, wd = flow.shape[:2]
        xx, yy = np.meshgrid(np.arange(wd), np.arange(ht))
        coords = np.stack([xx, yy], axis=-1).reshape(-1, 2).astype(np.float32)
        flow = flow.reshape(-1, 2).astype(np.float32)
        valid = valid.reshape(-1).astype(np.float32)
        keep = valid >= 1
        coords0, flow0 = coords[keep], flow[keep]
        ht1, wd1 = int(round(ht * fy)), int(round(wd * fx))
        coords1 = coords0 * [fx, fy]
        flow1 = flow0 * [fx, fy]
        xi = np.round(coords1[:, 0]).astype(np.int32)
        yi = np.round(coords1[:, 1]).astype(np.int32)
        v = (xi > 0) & (xi < wd1) & (yi > 0) & (yi < ht1)
        flow_img = np.zeros([ht1, wd1, 2], dtype=np.float32)
        valid_img = np.zeros([ht1, wd1], dtype=np.int32)
        flow_img[yi[v], xi[v]] = flow1[v]
        valid_img[yi[v], xi[v]] = 1
        return flow_img, valid_img

    def spatial_transform(self, img1, img2, flow, valid):
        ht, wd = img1.shape[:2]
        min_scale = np.maximum((self.crop_size[0] + 1) / float(ht), (self.crop_size[1] + 1) / float(wd))
        scale = 2 ** np.random.uniform(self.min_scale, self.max_scale)
        scale_x = np.clip(scale, min_scale, None)
        scale_y = np.clip(scale, min_scale, None)
        if np.random.rand() < self.spatial_aug_prob:
            img1 = resize_linear(img1, fx=scale_x, fy=scale_y)
            img2 = resize_linear(img2, fx=scale_x, fy=scale_y)
            flow, valid = self.resize_sparse_flow_map(flow, valid, fx=scale_x, fy=scale_y)
        if self.do_flip and np.random.rand() < 0.5:
            img1, img2 = img1[:, ::-1], img2[:, ::-1]
            flow = flow[:, ::-1] * [-1.0, 1.0]
            valid = valid[:, ::-1]
        margin_y, margin_x = 20, 50
        y0 = np.random.randint(0, img1.shape[0] - self.crop_size[0] + margin_y)
        x0 = np.random.randint(-margin_x, img1.shape[1] - self.crop_size[1] + margin_x)
        y0 = np.clip(y0, 0, img1.shape[0] - self.crop_size[0])
        x0 = np.clip(x0, 0, img1.shape[1] - self.crop_size[1])
        sl = (slice(y0, y0 + self.crop_size[0]), slice(x0, x0 + self.crop_size[1]))
        return img1[sl], img2[sl], flow[sl], valid[sl]

    def __call__(self, img1, img2, flow, valid):
        img1, img2 = self.color_transform(img1, img2)
        img1, img2 = self.eraser_transform(img1, img2)
        img1, img2, flow, valid = self.spatial_transform(img1, img2, flow, valid)
        return (np.ascontiguousarray(img1), np.ascontiguousarray(img2),
                np.ascontiguousarray(flow, dtype=np.float32), np.ascontiguousarray(valid))
