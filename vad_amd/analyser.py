"""Streaming analyser interface (reference realtime_analysis/analyser.py:4-15).

A plain class, as in the reference: the abstract markers are documentation
(the reference does not use ABCMeta, so abstractness is not enforced)."""
import abc


class Analyser:

    def __init__(self):
        pass

    @abc.abstractmethod
    def load_init_inactive_frames(self, frames):
        return

    @abc.abstractmethod
    def feed_frame(self, frame):
        return
