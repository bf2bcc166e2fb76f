"""Shared loaders for the golden fixtures extracted from the reference tests."""
import json
import os

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)["cases"]


def case_id(c):
    return c.get("source", "?").split("/")[-1] + ":" + c.get("name", "")[:40]
