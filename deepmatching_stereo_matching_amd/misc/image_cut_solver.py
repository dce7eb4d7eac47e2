"""ImageCutSolver mirror (reference: misc/image_cut_solver.py:26-197).

The reference solves its tiles one after another (``_execute_matching``, :163-175).  Here
all tiles go to the GPU as batches (engine.solve_tiles: one fused level-0/level-1 launch,
one launch per pyramid level and per matching level for the whole batch), and the
stitching -- later tiles overwrite earlier ones, j outer / i inner -- runs in dm_stitch.
Output cells no tile covers are NaN (``np.empty`` garbage in the reference).
"""

import numpy as np
import torch
from PIL import Image

from deepmatching_stereo_matching_amd import _lib as L
from deepmatching_stereo_matching_amd import engine


class ImageCutSolver():
    '''
    小画像に切ってそれぞれdeepmatchingに入れる
    '''

    def __init__(
        self, img1, img2,
        image_size=[32, 32], stride=[32, 32], window_size=5,
        feature_name='cv2.TM_CCOEFF_NORMED', degree_map_mode=['elevation'],
        padding=False,
        sub_pix=True,
        filtering=False,
        filtering_window_size=3,
        filtering_num=3,
        filtering_mode='average'
    ):
        self.img_shape = img1.shape
        assert self.img_shape == img2.shape, '2枚の画像は同じサイズ！'
        self.img1 = img1
        self.img2 = img2
        self.stride = stride
        self.window_size = window_size
        self.degree_map_mode = degree_map_mode
        self.exclusive_pix = int((window_size - 1) / 2)
        self.image_size = image_size
        self.trimed_size = [image_size[i] + 2 * self.exclusive_pix for i in range(2)]
        self.feature_name = feature_name
        if feature_name not in L.METHODS:
            from deepmatching_stereo_matching_amd.misc.Feature_value import Feature_value
            Feature_value(feature_name)  # prints + exits like the reference

        if padding:
            self._padding()

        # loop length
        self.len = [int(np.floor((self.img_shape[i] - self.trimed_size[i]) / self.stride[i])) for i in range(2)]

        self.padding = padding
        self.sub_pix = sub_pix
        self.filtering = filtering
        self.filtering_window_size = filtering_window_size
        self.filtering_num = filtering_num
        self.filtering_mode = filtering_mode

        self.log_flg = True

    def _padding(self):
        """Reproduces the reference exactly (:73-93): img1 is zero-padded by exclusive_pix
        (and copied in twice), img2 becomes all zeros of the padded size."""
        img1 = self.img1
        ex = self.exclusive_pix
        a = np.zeros([img1.shape[0] + 2 * ex, img1.shape[1] + 2 * ex])
        a[ex:-ex, ex:-ex] = img1
        self.img1 = a.astype(np.uint8)
        self.img2 = np.zeros(a.shape).astype(np.uint8)

    def _cut_and_pool(self):
        '''
        画像を切り出しリストで保存 (crops are views; the batched solver uses the origins)
        '''
        self.img1_sub = []
        self.img2_sub = []
        self.img_index = []
        for j in range(self.len[1]):
            for i in range(self.len[0]):
                r, c = self.stride[0] * i, self.stride[1] * j
                self.img1_sub.append(self.img1[r:r + self.trimed_size[0], c:c + self.trimed_size[1]])
                self.img2_sub.append(self.img2[r:r + self.trimed_size[0], c:c + self.trimed_size[1]])
                self.img_index.append([i, j])

    def _solver(self, solve_image, solve_template):
        """
        小画像に対しdeepmatchingを実施する: one (S+2e)^2 crop pair -> (d_maps, score map),
        as the reference's _solver (:115-142) returns them; solved by the same batched device
        path as _execute_matching (a batch of one tile).
        """
        h0 = np.shape(solve_image)[0] - 2 * self.exclusive_pix
        w0 = np.shape(solve_image)[1] - 2 * self.exclusive_pix
        self._log_pyramid(h0, w0)
        match = engine.solve_tiles(solve_image, solve_template, [[0, 0]], h0, w0, self.window_size,
                                   L.METHODS[self.feature_name], self.sub_pix, self.filtering,
                                   self.filtering_window_size, self.filtering_num,
                                   self.filtering_mode)[0]
        d = np.array([engine.cal_map(match, m).cpu().numpy() for m in self.degree_map_mode])
        return d, match[2].cpu().numpy()

    def _log_pyramid(self, h0, w0):
        if self.log_flg:
            nlev, N = engine.pyramid_plan(h0, w0)
            print('complete to create multi-level correlation pyramid')
            print('pyramid level: {}, N={}'.format(nlev, N))
            self.log_flg = False

    def _execute_matching_device(self):
        """All tiles in batches on the GPU -> (d_map, out_map) device tensors.  The tile grid
        is self.len, counted on the image shape BEFORE _padding (:46,58-62).  Opted in to tile
        sharding (shard.tile_sharding() or DM_SHARD_TILES=1) under a torch.distributed process
        group, the tiles are sharded over its ranks by shard.BandSolver -- the path bench.py's
        c5_split line measures: rank r solves one contiguous band of tiles in chunks, each
        chunk's results gathered to rank 0 behind the compute, rank 0 stitches -- and the maps
        come back on every rank (one broadcast; tile_sharding(result='root'): rank 0 only, the
        others get None).  Every rank must then solve the same pair (shard.broadcast_pair
        sends it from rank 0)."""
        from deepmatching_stereo_matching_amd import shard
        n = list(self.len)
        if n[0] < 1 or n[1] < 1:
            raise IndexError('list index out of range')   # img_index[-1] of an empty cut (:150)
        origins = np.array([(self.stride[0] * i, self.stride[1] * j)
                            for j in range(n[1]) for i in range(n[0])], dtype=np.int64)
        h0, w0 = self.image_size
        self._log_pyramid(h0, w0)
        args = (self.img1, self.img2, origins, h0, w0, self.window_size,
                L.METHODS[self.feature_name], self.sub_pix, self.filtering,
                self.filtering_window_size, self.filtering_num, self.filtering_mode)
        if shard.tile_sharding_enabled():
            return shard.solve_image_sharded(self.img1, self.img2, [h0, w0], self.stride, self.window_size,
                                             L.METHODS[self.feature_name], self.degree_map_mode,
                                             self.sub_pix, self.filtering, self.filtering_window_size,
                                             self.filtering_num, self.filtering_mode,
                                             result=shard.shard_result(), grid=(n, origins))
        match = engine.solve_tiles(*args)
        return engine.stitch(match, n, h0, w0, self.stride, self.degree_map_mode)

    def _execute_matching(self):
        """
        小画像ごとにマッチングを行い結果を結合
        """
        d_map, out_map = self._execute_matching_device()
        # (None on the ranks other than 0 of a sharded solve with tile_sharding(result='root'))
        self.d_map = d_map.cpu().numpy() if d_map is not None else None
        self.out_map = out_map.cpu().numpy() if out_map is not None else None

    def __call__(self):
        self._cut_and_pool()
        self._execute_matching()
        return self.d_map, self.out_map

    @staticmethod
    def image_save(path, arr, threshold=[100, 190]):
        """
        numpy配列を画像として保存 (clamped to threshold, uint8 PNG)
        """
        arr = np.where(arr > threshold[1], threshold[1], arr)
        arr = np.where(arr < threshold[0], threshold[0], arr)
        pil_img = Image.fromarray(arr.astype(np.uint8))
        pil_img.save(path)
