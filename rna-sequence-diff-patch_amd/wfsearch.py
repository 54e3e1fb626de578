"""Batched one-vs-many Wagner-Fischer search.

The reference scores a query against every document of the collection with one full
`wagnerFisher` per pair (`IRMethods.search_collection`, IRMethods.py:443-477, method
`wf_score`, :435-440), and `create_search_threads` runs that search twice per query
(:487-491 and :511-515).  Here the whole collection is one engine launch (short piRNA
documents go to the lane-per-pair kernel), and repeated searches with the same query,
documents and cost table are answered from a small cache.

    search_collection(query, vector_type, collection, wf_score, return_dict=None, callback=None)

has the reference's signature and output: a list of (doc['sequence'], score) in
`collection.find({})` order, delivered through callback / return_dict['wf_score'] /
the return value exactly like the reference.  Other scoring methods (tf/idf vectors, set
similarities) are not on the engine's path and raise NotImplementedError.
"""
from collections import OrderedDict

import StringEditDistance as SED

_CACHE = OrderedDict()
_CACHE_SIZE = 8


def wf_score(seq1, seq2, user_cost=False):
    """IRMethods.wf_score (IRMethods.py:435-440): 1 / (1 + dp[n][m].value)."""
    dp = SED.wagnerFisher(seq1, seq2, user_cost)
    cost = dp[len(dp) - 1][len(dp[0]) - 1].value
    return 1 / (1 + cost)


def wf_scores(query, seqs, user_cost=False):
    """[wf_score(query, s, user_cost) for s in seqs] with one engine launch (cached)."""
    seqs = list(seqs)
    if not seqs:
        return []
    queries = [query] * len(seqs)
    plan = SED.batch_plan(queries, seqs, user_cost)  # the reference raises on the first offending document, in order
    key = (query, tuple(seqs), plan.key())
    hit = _CACHE.get(key)
    if hit is not None:
        _CACHE.move_to_end(key)
        return list(hit)
    vals = SED.distance_batch(queries, seqs, user_cost, plan=plan)
    scores = [1 / (1 + v) for v in vals]
    _CACHE[key] = tuple(scores)
    while len(_CACHE) > _CACHE_SIZE:
        _CACHE.popitem(last=False)
    return scores


def clear_cache():
    _CACHE.clear()


def search_collection(query, vector_type, collection, method, return_dict=None, callback=None):
    """IRMethods.search_collection for method == wf_score (IRMethods.py:443-477)."""
    if getattr(method, '__name__', None) != 'wf_score':
        raise NotImplementedError("only the wf_score method runs on the edit-distance engine")
    seqs = [doc['sequence'] for doc in collection.find({})]
    scores = list(zip(seqs, wf_scores(query, seqs)))
    if callback is not None:
        callback(scores)
    elif return_dict is not None:
        return_dict[method.__name__] = scores
    else:
        return scores
