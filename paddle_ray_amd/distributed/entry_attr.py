"""Sparse-table entry policies (parity: python/paddle/distributed/entry_attr.py)."""


class EntryAttr:
    def _to_attr(self):
        raise NotImplementedError


class ProbabilityEntry(EntryAttr):
    def __init__(self, probability):
        self._name, self._probability = 'probability_entry', probability

    def _to_attr(self):
        return f'{self._name}:{self._probability}'


class CountFilterEntry(EntryAttr):
    def __init__(self, count_filter):
        self._name, self._count_filter = 'count_filter_entry', count_filter

    def _to_attr(self):
        return f'{self._name}:{self._count_filter}'


class ShowClickEntry(EntryAttr):
    def __init__(self, show_name, click_name):
        self._name, self._show, self._click = 'show_click_entry', show_name, click_name

    def _to_attr(self):
        return f'{self._name}:{self._show}:{self._click}'
