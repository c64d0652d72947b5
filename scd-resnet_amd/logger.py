"""ANSI-coloured console logging and a tqdm-safe stdout redirect (logger.py of the reference)."""
import contextlib
import sys

from tqdm import tqdm

_RESET = "\033[0m"
_COLORS = {"black": "\033[30m", "red": "\033[31m", "green": "\033[32m", "yellow": "\033[33m",
           "blue": "\033[34m", "purple": "\033[35m", "darkgreen": "\033[36m", "white": "\033[37m"}


class Logger:
    CLEARSTYLES = _RESET

    @staticmethod
    def _emit(color, msg):
        print(_COLORS[color] + msg + _RESET)

    info = staticmethod(lambda msg: Logger._emit("blue", msg))
    infoGreen = staticmethod(lambda msg: Logger._emit("green", msg))
    warn = staticmethod(lambda msg: Logger._emit("yellow", msg))
    err = staticmethod(lambda msg: Logger._emit("red", msg))

    @staticmethod
    def log(msg):
        print(_RESET + msg)


class TqdmFile(object):
    def __init__(self, textIO):
        self.textIO = textIO

    def write(self, x):
        if x.rstrip():
            tqdm.write(x, file=self.textIO)

    def flush(self):
        self.textIO.flush()


@contextlib.contextmanager
def monitorStdOutStream():
    saved = sys.stdout
    try:
        sys.stdout = TqdmFile(saved)
        yield saved
    finally:
        sys.stdout = saved
