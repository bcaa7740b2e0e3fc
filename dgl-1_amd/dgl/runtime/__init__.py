"""Scheduler and executors of the message-passing API."""
from __future__ import absolute_import

from . import ir, runtime, scheduler, spmv, degree_bucketing  # noqa: F401
