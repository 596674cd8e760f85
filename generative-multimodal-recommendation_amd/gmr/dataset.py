"""Interaction dataset + split — mirrors utils/dataset.py of the reference.

Input format (reference utils/dataset.py:50-63): a TSV `<data_path><dataset>/<inter_file_name>`
with columns USER_ID_FIELD, ITEM_ID_FIELD, the splitting label (0 train / 1 valid / 2 test)
and an optional rating column.  user_num / item_num = max id + 1 (:47-48).  Cold users of the
valid/test splits are dropped when filter_out_cod_start_users (:65-82).
A dataset may also be built in memory (synthetic benchmark data) and carry its modality
features (`v_feat` / `t_feat` numpy arrays) instead of .npy files.
"""
import os

import numpy as np
import pandas as pd


class RecDataset:
    def __init__(self, config, df=None):
        self.config = config
        self.dataset_name = config["dataset"]
        self.dataset_path = os.path.abspath((config["data_path"] or "") + (self.dataset_name or ""))
        self.uid_field = config["USER_ID_FIELD"]
        self.iid_field = config["ITEM_ID_FIELD"]
        self.splitting_label = config["inter_splitting_label"]
        self.v_feat = None
        self.t_feat = None
        if df is not None:
            self.df = df
            return
        f = os.path.join(self.dataset_path, config["inter_file_name"])
        if not os.path.isfile(f):
            raise ValueError(f"File {f} not exist")
        self.rating_field = config["RATING_FIELD"] if "RATING_FIELD" in config else None
        cols = [self.uid_field, self.iid_field, self.splitting_label]
        if self.rating_field:
            cols.append(self.rating_field)
        self.df = pd.read_csv(f, usecols=cols, sep=config["field_separator"])
        self.item_num = int(self.df[self.iid_field].max()) + 1
        self.user_num = int(self.df[self.uid_field].max()) + 1

    @classmethod
    def from_arrays(cls, config, users, items, labels, user_num=None, item_num=None, v_feat=None, t_feat=None):
        df = pd.DataFrame({config["USER_ID_FIELD"]: np.asarray(users, np.int64),
                           config["ITEM_ID_FIELD"]: np.asarray(items, np.int64),
                           config["inter_splitting_label"]: np.asarray(labels, np.int64)})
        ds = cls(config, df)
        ds.user_num = int(user_num if user_num is not None else df[config["USER_ID_FIELD"]].max() + 1)
        ds.item_num = int(item_num if item_num is not None else df[config["ITEM_ID_FIELD"]].max() + 1)
        ds.v_feat, ds.t_feat = v_feat, t_feat
        return ds

    def split(self):
        parts = []
        for lb in range(3):
            d = self.df[self.df[self.splitting_label] == lb].drop(columns=[self.splitting_label])
            parts.append(d)
        if self.config["filter_out_cod_start_users"]:
            train_u = set(parts[0][self.uid_field].values.tolist())
            for i in (1, 2):
                parts[i] = parts[i][parts[i][self.uid_field].isin(train_u)]
        return [self.copy(p) for p in parts]

    def copy(self, new_df):
        nxt = RecDataset(self.config, new_df)
        nxt.item_num, nxt.user_num = self.item_num, self.user_num
        nxt.v_feat, nxt.t_feat = self.v_feat, self.t_feat
        return nxt

    def get_user_num(self):
        return self.user_num

    def get_item_num(self):
        return self.item_num

    def shuffle(self):
        self.df = self.df.sample(frac=1, replace=False).reset_index(drop=True)

    def __len__(self):
        return len(self.df)

    def __getitem__(self, idx):
        return self.df.iloc[idx]

    def __str__(self):
        self.inter_num = len(self.df)
        info = [str(self.dataset_name)]
        nu = self.df[self.uid_field].nunique()
        ni = self.df[self.iid_field].nunique()
        if nu:
            info += [f"The number of users: {nu}", f"Average actions of users: {self.inter_num / nu}"]
        if ni:
            info += [f"The number of items: {ni}", f"Average actions of items: {self.inter_num / ni}"]
        info.append(f"The number of inters: {self.inter_num}")
        if nu and ni:
            info.append(f"The sparsity of the dataset: {(1 - self.inter_num / nu / ni) * 100}%")
        return "\n".join(info)

    __repr__ = __str__
