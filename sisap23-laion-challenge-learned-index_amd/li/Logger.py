"""Logger mixin (reference search/li/Logger.py:4-18): same format string."""
import logging


class Logger:
    @property
    def logger(self):
        logging.basicConfig(
            level=logging.INFO,
            format='[%(asctime)s][%(levelname)-5.5s][%(name)-.20s] %(message)s')
        return logging.getLogger(self.__class__.__name__)
