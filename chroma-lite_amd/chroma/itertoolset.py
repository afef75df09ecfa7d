"""Iterator helpers used by the simulation driver (reference chroma/itertoolset.py)."""
from itertools import chain, cycle, islice


def peek(iterable):
    """(first_element, equivalent_iterator)."""
    it = iter(iterable)
    first = next(it)
    return first, chain([first], it)


def roundrobin(*iterables):
    """roundrobin('ABC', 'D', 'EF') --> A D E B F C"""
    pending = len(iterables)
    nexts = cycle(iter(it).__next__ for it in iterables)
    while pending:
        try:
            for nxt in nexts:
                yield nxt()
        except StopIteration:
            pending -= 1
            nexts = cycle(islice(nexts, pending))


def flatten(list_of_lists):
    return chain.from_iterable(list_of_lists)
