"""Logging setup — same stream/file format as utils/logger.py of the reference (:13-63)."""
import logging
import os

from .utils import get_local_time


def init_logger(config, log_dir="./log/"):
    """Under data parallelism only rank 0 writes the log file (and logs at the configured
    level); the other ranks log warnings and errors to the stream."""
    from . import dist
    state = (config["state"] or "info").lower()
    level = {"debug": logging.DEBUG, "error": logging.ERROR, "warning": logging.WARNING,
             "critical": logging.CRITICAL}.get(state, logging.INFO)
    if dist.rank() != 0:
        sh = logging.StreamHandler()
        sh.setLevel(logging.WARNING)
        sh.setFormatter(logging.Formatter("%(asctime)-15s rank" + str(dist.rank()) + " %(levelname)s %(message)s",
                                          "%d %b %H:%M"))
        logging.basicConfig(level=logging.WARNING, handlers=[sh], force=True)
        return None
    os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, "{}-{}-{}.log".format(config["model"], config["dataset"], get_local_time()))
    fh = logging.FileHandler(path, "w", "utf-8")
    fh.setLevel(level)
    fh.setFormatter(logging.Formatter("%(asctime)-15s %(levelname)s %(message)s", "%a %d %b %Y %H:%M:%S"))
    sh = logging.StreamHandler()
    sh.setLevel(level)
    sh.setFormatter(logging.Formatter("%(asctime)-15s %(levelname)s %(message)s", "%d %b %H:%M"))
    logging.basicConfig(level=level, handlers=[sh, fh], force=True)
    return path
