"""quick_start — mirrors utils/quick_start.py of the reference (config -> data -> grid -> fit).

config_dict may carry `synthetic: <shape>` (gmr.synthetic.SHAPES) to generate an Amazon-shaped
dataset in memory instead of reading <data_path>/<dataset>/<inter_file_name>.
"""
import os
import platform
from itertools import product
from logging import getLogger

from .configurator import Config
from .dataloader import EvalDataLoader, TrainDataLoader
from .dataset import RecDataset
from .logger import init_logger
from .utils import dict2str, get_model, get_trainer, init_seed


def build_data(config):
    if config["synthetic"]:
        from .synthetic import make_dataset
        dataset = make_dataset(config, config["synthetic"], seed=int(config["synthetic_seed"] or 0))
    else:
        dataset = RecDataset(config)
    return dataset


def popularity_groups(config, train_dataset):
    """Popular items (top 20 % by train count) and warm users (> 5 train interactions), quick_start.py:46-102."""
    iid, uid = config["ITEM_ID_FIELD"], config["USER_ID_FIELD"]
    df = train_dataset.df
    items = df[iid].value_counts().index.tolist()
    pop_items = set(items[:int(len(items) * 0.2)])
    uc = df[uid].value_counts()
    warm = set(uc[uc > 5].index.tolist())
    return pop_items, warm, len(items), len(uc)


def quick_start(model, dataset, config_dict, save_model=True, mg=False):
    config = Config(model, dataset, config_dict, mg)
    init_logger(config)
    logger = getLogger()
    logger.info("██Server: \t" + platform.node())
    logger.info("██Dir: \t" + os.getcwd() + "\n")
    logger.info(config)
    ds = build_data(config)
    logger.info(str(ds))
    train_ds, valid_ds, test_ds = ds.split()
    logger.info("\n====Training====\n" + str(train_ds))
    logger.info("\n====Validation====\n" + str(valid_ds))
    logger.info("\n====Testing====\n" + str(test_ds))
    pop_items, warm, n_items_tr, n_users_tr = popularity_groups(config, train_ds)
    config["pop_items"] = pop_items
    config["warm_users"] = warm
    logger.info(f"Train dataset All Interaction items count: {n_items_tr}, Popular items count: {len(pop_items)}, "
                f"Niche items count: {n_items_tr - len(pop_items)}")
    logger.info("User Grouping based on Training History (Threshold=5):")
    logger.info(f"  Warm Users (>5 interactions): {len(warm)}")
    logger.info(f"  Cold Users (<=5 interactions): {n_users_tr - len(warm)} (in training set)")
    train_data = TrainDataLoader(config, train_ds, batch_size=config["train_batch_size"], shuffle=True)
    valid_data = EvalDataLoader(config, valid_ds, additional_dataset=train_ds, batch_size=config["eval_batch_size"])
    test_data = EvalDataLoader(config, test_ds, additional_dataset=train_ds, batch_size=config["eval_batch_size"])
    logger.info("\n\n=================================\n\n")
    hyper = list(config["hyper_parameters"])
    if "seed" not in hyper:
        hyper = ["seed"] + hyper
    combos = list(product(*[config[i] or [None] for i in hyper]))
    val_metric = config["valid_metric"].lower()
    results, best_idx, best_val = [], 0, 0.0
    for idx, tup in enumerate(combos):
        for k, v in zip(hyper, tup):
            config[k] = v
        init_seed(config["seed"])
        logger.info("========={}/{}: Parameters:{}={}=======".format(idx + 1, len(combos), hyper, tup))
        train_data.pretrain_setup()
        m = get_model(config["model"])(config, train_data)
        logger.info(m)
        trainer = get_trainer(config["model"])(config, m, mg)
        best_valid_score, best_valid, best_test = trainer.fit(train_data, valid_data=valid_data, test_data=test_data,
                                                              saved=save_model)
        results.append((tup, best_valid, best_test))
        if best_test[val_metric] > best_val:
            best_val, best_idx = best_test[val_metric], idx
        logger.info("best valid result: {}".format(dict2str(best_valid)))
        logger.info("test result: {}".format(dict2str(best_test)))
        logger.info("████Current BEST████:\nParameters: {}={},\nValid: {},\nTest: {}\n\n\n".format(
            hyper, results[best_idx][0], dict2str(results[best_idx][1]), dict2str(results[best_idx][2])))
    logger.info("\n============All Over=====================")
    for p, k, v in results:
        logger.info("Parameters: {}={},\n best valid: {},\n best test: {}".format(hyper, p, dict2str(k), dict2str(v)))
    logger.info("\n\n█████████████ BEST ████████████████")
    logger.info("\tParameters: {}={},\nValid: {},\nTest: {}\n\n".format(
        hyper, results[best_idx][0], dict2str(results[best_idx][1]), dict2str(results[best_idx][2])))
    return results
