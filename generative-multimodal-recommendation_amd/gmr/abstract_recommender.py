"""Model base classes — mirror common/abstract_recommender.py of the reference.

GeneralRecommender(config, dataloader) reads n_users / n_items from the dataloader's dataset
and loads the modality features (image/text) as fp32 device tensors
(reference abstract_recommender.py:75-103).  Feature files are read with numpy's safe
loader (allow_pickle=False); in-memory datasets may carry the arrays directly.
"""
import os

import numpy as np
import torch
import torch.nn as nn


class AbstractRecommender(nn.Module):
    def pre_epoch_processing(self):
        pass

    def post_epoch_processing(self):
        pass

    def calculate_loss(self, interaction):
        raise NotImplementedError

    def predict(self, interaction):
        raise NotImplementedError

    def full_sort_predict(self, interaction):
        raise NotImplementedError

    def __str__(self):
        n = sum(int(np.prod(p.size())) for p in self.parameters())
        return super().__str__() + "\nTrainable parameters: {}".format(n)


class GeneralRecommender(AbstractRecommender):
    def __init__(self, config, dataloader):
        super().__init__()
        self.USER_ID = config["USER_ID_FIELD"]
        self.ITEM_ID = config["ITEM_ID_FIELD"]
        self.NEG_ITEM_ID = (config["NEG_PREFIX"] or "neg__") + (self.ITEM_ID or "")
        self.n_users = dataloader.dataset.get_user_num()
        self.n_items = dataloader.dataset.get_item_num()
        self.batch_size = config["train_batch_size"]
        self.device = config["device"]
        self.v_feat, self.t_feat = None, None
        if not config["end2end"] and config["is_multimodal_model"]:
            ds = dataloader.dataset
            v = getattr(ds, "v_feat", None)
            t = getattr(ds, "t_feat", None)
            if v is None and t is None:
                path = os.path.abspath((config["data_path"] or "") + (config["dataset"] or ""))
                vf = os.path.join(path, config["vision_feature_file"] or "")
                tf = os.path.join(path, config["text_feature_file"] or "")
                if os.path.isfile(vf):
                    v = np.load(vf, allow_pickle=False)
                if os.path.isfile(tf):
                    t = np.load(tf, allow_pickle=False)
            if v is not None:
                self.v_feat = torch.as_tensor(np.asarray(v, np.float32)).to(self.device)
            if t is not None:
                self.t_feat = torch.as_tensor(np.asarray(t, np.float32)).to(self.device)
            assert self.v_feat is not None or self.t_feat is not None, "Features all NONE"
