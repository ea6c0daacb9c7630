"""Classic NLP datasets (parity: python/paddle/text/datasets/*.py). Nothing is downloaded
here: every dataset reads the public archive from ``data_file`` (the same file the
reference would have downloaded), parsed in the same way."""
import collections
import re
import string
import tarfile
import zipfile

import numpy as np

from ...io import Dataset


def _need(data_file, name):
    if data_file is None:
        raise ValueError(f"{name}: automatic download is unavailable in this environment; "
                         f"pass data_file=<path to the archive>")
    return data_file


class UCIHousing(Dataset):
    """Boston housing regression: 13 normalised features -> price (80/20 train/test)."""

    def __init__(self, data_file=None, mode='train', download=True):
        if mode.lower() not in ('train', 'test'):
            raise ValueError(f"mode should be 'train' or 'test', but got {mode}")
        self.mode = mode.lower()
        self.data_file = _need(data_file, 'UCIHousing')
        data = np.fromfile(self.data_file, sep=' ')
        fn = 14
        data = data.reshape(data.shape[0] // fn, fn)
        mx, mn, avg = data.max(0), data.min(0), data.sum(0) / data.shape[0]
        for i in range(fn - 1):
            data[:, i] = (data[:, i] - avg[i]) / (mx[i] - mn[i])
        off = int(data.shape[0] * 0.8)
        self.data = data[:off] if self.mode == 'train' else data[off:]
        from ...framework.core import get_default_dtype
        self.dtype = str(get_default_dtype()).replace('torch.', '')

    def __getitem__(self, idx):
        d = self.data[idx]
        return np.array(d[:-1]).astype(self.dtype), np.array(d[-1:]).astype(self.dtype)

    def __len__(self):
        return len(self.data)


def _tokenize_tar(path, pattern):
    docs = []
    with tarfile.open(path) as tf:
        for m in tf:
            if pattern.match(m.name):
                raw = tf.extractfile(m).read().rstrip(b'\n\r')
                docs.append(raw.translate(None, string.punctuation.encode('latin-1'))
                            .lower().split())
    return docs


class Imdb(Dataset):
    """IMDB sentiment (aclImdb_v1.tar.gz): word-id docs, label 0 = pos, 1 = neg."""

    def __init__(self, data_file=None, mode='train', cutoff=150, download=True):
        if mode.lower() not in ('train', 'test'):
            raise ValueError(f"mode should be 'train', 'test', but got {mode}")
        self.mode = mode.lower()
        self.data_file = _need(data_file, 'Imdb')
        freq = collections.defaultdict(int)
        for doc in _tokenize_tar(self.data_file,
                                 re.compile(r"aclImdb/((train)|(test))/((pos)|(neg))/.*\.txt$")):
            for w in doc:
                freq[w] += 1
        items = sorted([x for x in freq.items() if x[1] > cutoff], key=lambda x: (-x[1], x[0]))
        self.word_idx = {w: i for i, (w, _) in enumerate(items)}
        self.word_idx['<unk>'] = len(items)
        unk = self.word_idx['<unk>']
        self.docs, self.labels = [], []
        for lab, pol in ((0, 'pos'), (1, 'neg')):
            pat = re.compile(rf"aclImdb/{self.mode}/{pol}/.*\.txt$")
            for doc in _tokenize_tar(self.data_file, pat):
                self.docs.append([self.word_idx.get(w, unk) for w in doc])
                self.labels.append(lab)

    def __getitem__(self, idx):
        return np.array(self.docs[idx]), np.array([self.labels[idx]])

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    """PTB language-model data (simple-examples.tgz): 'NGRAM' windows or 'SEQ' (src, trg)."""

    def __init__(self, data_file=None, data_type='NGRAM', window_size=-1, mode='train',
                 min_word_freq=50, download=True):
        if data_type.upper() not in ('NGRAM', 'SEQ'):
            raise ValueError("data type should be 'NGRAM', 'SEQ'")
        self.data_type = data_type.upper()
        if mode.lower() not in ('train', 'test'):
            raise ValueError("mode should be 'train', 'test'")
        self.mode = mode.lower()
        self.window_size, self.min_word_freq = window_size, min_word_freq
        self.data_file = _need(data_file, 'Imikolov')
        with tarfile.open(self.data_file) as tf:
            trainf = tf.extractfile('./simple-examples/data/ptb.train.txt')
            testf = tf.extractfile('./simple-examples/data/ptb.valid.txt')
            train_lines, test_lines = trainf.readlines(), testf.readlines()
        freq = collections.defaultdict(int)
        for lines in (train_lines, test_lines):
            for ln in lines:
                for w in ln.strip().split():
                    freq[w] += 1
                freq[b'<s>'] += 1
                freq[b'<e>'] += 1
        freq.pop(b'<unk>', None)
        items = sorted([x for x in freq.items() if x[1] > min_word_freq],
                       key=lambda x: (-x[1], x[0]))
        self.word_idx = {w: i for i, (w, _) in enumerate(items)}
        self.word_idx[b'<unk>'] = len(items)
        unk = self.word_idx[b'<unk>']
        self.data = []
        for ln in (train_lines if self.mode == 'train' else test_lines):
            if self.data_type == 'NGRAM':
                if self.window_size < 0:
                    raise ValueError("NGRAM needs window_size > 0")
                ids = [self.word_idx.get(w, unk) for w in [b'<s>'] + ln.strip().split() +
                       [b'<e>']]
                if len(ids) >= self.window_size:
                    for i in range(self.window_size, len(ids) + 1):
                        self.data.append(tuple(ids[i - self.window_size:i]))
            else:
                ids = [self.word_idx.get(w, unk) for w in ln.strip().split()]
                src = [self.word_idx[b'<s>']] + ids
                trg = ids + [self.word_idx[b'<e>']]
                if self.window_size > 0 and len(src) > self.window_size:
                    continue
                self.data.append((src, trg))

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


class Movielens(Dataset):
    """MovieLens-1M (ml-1m.zip): (user id, gender, age, job, movie id, categories, title
    ids, rating) records, a deterministic ``test_ratio`` split by ``rand_seed``."""

    def __init__(self, data_file=None, mode='train', test_ratio=0.1, rand_seed=0,
                 download=True):
        if mode.lower() not in ('train', 'test'):
            raise ValueError("mode should be 'train', 'test'")
        self.mode = mode.lower()
        self.data_file = _need(data_file, 'Movielens')
        rng = np.random.RandomState(rand_seed)
        pat = re.compile(r'^(.*)\((\d+)\)$')
        self.movie_info, self.user_info = {}, {}
        title_words, cats = set(), set()
        age_table = [1, 18, 25, 35, 45, 50, 56]
        with zipfile.ZipFile(self.data_file) as z:
            for ln in z.read('ml-1m/movies.dat').decode('latin-1').splitlines():
                mid, title, cat = ln.strip().split('::')
                c = cat.split('|')
                cats.update(c)
                t = pat.match(title).group(1).lower().split() if pat.match(title) else \
                    title.lower().split()
                title_words.update(t)
                self.movie_info[int(mid)] = (int(mid), c, t)
            self.cat_dict = {c: i for i, c in enumerate(sorted(cats))}
            self.title_dict = {w: i for i, w in enumerate(sorted(title_words))}
            for ln in z.read('ml-1m/users.dat').decode('latin-1').splitlines():
                uid, gender, age, job, _ = ln.strip().split('::')
                self.user_info[int(uid)] = (int(uid), 0 if gender == 'M' else 1,
                                            age_table.index(int(age)), int(job))
            self.data = []
            for ln in z.read('ml-1m/ratings.dat').decode('latin-1').splitlines():
                is_test = rng.random_sample() < test_ratio
                if is_test != (self.mode == 'test'):
                    continue
                uid, mid, rating, _ = ln.strip().split('::')
                u = self.user_info[int(uid)]
                m = self.movie_info[int(mid)]
                self.data.append([[u[0]], [u[1]], [u[2]], [u[3]], [m[0]],
                                  [self.cat_dict[c] for c in m[1]],
                                  [self.title_dict[w] for w in m[2]],
                                  [float(rating) * 2 - 5.0]])

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


class _ParallelCorpus(Dataset):
    """Tokenised parallel text from a tar archive: ``(src_ids, trg_ids, trg_ids_next)``
    with <s>=0, <e>=1, <unk>=2 and dictionaries built from the training split (the
    WMT14/16 data layout: ``<split>/<lang>`` files or tab-separated ``src\\ttrg`` lines)."""

    START, END, UNK = '<s>', '<e>', '<unk>'

    def _build(self, pairs, src_dict_size, trg_dict_size):
        def vocab(seqs, size):
            c = collections.Counter(w for s in seqs for w in s)
            words = [w for w, _ in sorted(c.items(), key=lambda x: (-x[1], x[0]))]
            words = words[:max(0, size - 3)] if size > 0 else words
            return {w: i + 3 for i, w in enumerate(words)} | \
                {self.START: 0, self.END: 1, self.UNK: 2}
        self.src_dict = vocab([p[0] for p in pairs], src_dict_size)
        self.trg_dict = vocab([p[1] for p in pairs], trg_dict_size)

    def _encode(self, pairs):
        self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
        for s, t in pairs:
            si = [self.src_dict.get(w, 2) for w in [self.START] + s + [self.END]]
            ti = [self.trg_dict.get(w, 2) for w in t]
            self.src_ids.append(si)
            self.trg_ids.append([0] + ti)
            self.trg_ids_next.append(ti + [1])

    def __getitem__(self, idx):
        return (np.array(self.src_ids[idx]), np.array(self.trg_ids[idx]),
                np.array(self.trg_ids_next[idx]))

    def __len__(self):
        return len(self.src_ids)

    def get_dict(self, reverse=False):
        if reverse:
            return ({v: k for k, v in self.src_dict.items()},
                    {v: k for k, v in self.trg_dict.items()})
        return self.src_dict, self.trg_dict

    @staticmethod
    def _read_pairs(path, member_filter):
        pairs = []
        with tarfile.open(path) as tf:
            for m in tf:
                if m.isfile() and member_filter(m.name):
                    for ln in tf.extractfile(m).read().decode('utf-8', 'ignore').splitlines():
                        if '\t' in ln:
                            s, t = ln.split('\t')[:2]
                            pairs.append((s.split(), t.split()))
        return pairs


class WMT14(_ParallelCorpus):
    def __init__(self, data_file=None, mode='train', dict_size=-1, download=True):
        if mode.lower() not in ('train', 'test', 'gen'):
            raise ValueError("mode should be 'train', 'test' or 'gen'")
        self.mode = mode.lower()
        self.data_file = _need(data_file, 'WMT14')
        train = self._read_pairs(self.data_file, lambda n: '/train/' in n or
                                 n.endswith('train'))
        self._build(train, dict_size, dict_size)
        cur = train if self.mode == 'train' else self._read_pairs(
            self.data_file, lambda n: f'/{self.mode}/' in n or n.endswith(self.mode))
        self._encode(cur)


class WMT16(_ParallelCorpus):
    def __init__(self, data_file=None, mode='train', src_dict_size=-1, trg_dict_size=-1,
                 lang='en', download=True):
        if mode.lower() not in ('train', 'test', 'val'):
            raise ValueError("mode should be 'train', 'test' or 'val'")
        self.mode, self.lang = mode.lower(), lang
        self.data_file = _need(data_file, 'WMT16')
        train = self._read_pairs(self.data_file, lambda n: 'train' in n.split('/')[-1])
        if lang != 'en':
            train = [(t, s) for s, t in train]
        self._build(train, src_dict_size, trg_dict_size)
        cur = train if self.mode == 'train' else self._read_pairs(
            self.data_file, lambda n: self.mode in n.split('/')[-1])
        if self.mode != 'train' and lang != 'en':
            cur = [(t, s) for s, t in cur]
        self._encode(cur)


class Conll05st(Dataset):
    """CoNLL-2005 SRL test set (conll05st-tests.tar.gz + word/verb/target dicts + embedding):
    per predicate a (word, ctx_n2, ctx_n1, ctx_0, ctx_p1, ctx_p2, pred, mark, label)
    sample of id sequences."""

    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None,
                 target_dict_file=None, emb_file=None, download=True):
        self.data_file = _need(data_file, 'Conll05st')
        for f, n in ((word_dict_file, 'word_dict_file'), (verb_dict_file, 'verb_dict_file'),
                     (target_dict_file, 'target_dict_file')):
            _need(f, f'Conll05st {n}')
        self.emb_file = emb_file
        load = lambda p: {ln.strip(): i for i, ln in enumerate(open(p))}  # noqa: E731
        self.word_dict = load(word_dict_file)
        self.predicate_dict = load(verb_dict_file)
        self.label_dict = load(target_dict_file)
        self._load_anno()

    def _load_anno(self):
        sentences, labels = [], []
        with tarfile.open(self.data_file) as tf:
            words_f = [m for m in tf if m.name.endswith('test.wsj.words.gz')]
            props_f = [m for m in tf if m.name.endswith('test.wsj.props.gz')]
            if not words_f or not props_f:
                raise ValueError("Conll05st: archive lacks test.wsj.words.gz / props.gz")
            import gzip
            words = gzip.decompress(tf.extractfile(words_f[0]).read()).decode().splitlines()
            props = gzip.decompress(tf.extractfile(props_f[0]).read()).decode().splitlines()
        sent, lab = [], []
        for w, p in zip(words, props):
            if not w.strip():
                if sent:
                    sentences.append(sent)
                    labels.append(lab)
                sent, lab = [], []
                continue
            sent.append(w.strip())
            lab.append(p.strip().split())
        self.samples = []
        unk = self.word_dict.get('<unk>', 0)
        for sent, lab in zip(sentences, labels):
            cols = list(zip(*lab)) if lab else []
            if not cols:
                continue
            verbs = cols[0]
            for k, col in enumerate(cols[1:]):
                vidx = [i for i, v in enumerate(verbs) if v != '-']
                if k >= len(vidx):
                    break
                vi = vidx[k]
                tags, cur = [], 'O'
                for c in col:
                    if c.startswith('('):
                        cur = c.strip('()*')
                        tags.append('B-' + cur)
                        if c.endswith(')'):
                            cur = 'O'
                    elif cur != 'O':
                        tags.append('I-' + cur)
                        if c.endswith(')'):
                            cur = 'O'
                    else:
                        tags.append('O')
                wid = [self.word_dict.get(w, unk) for w in sent]
                ctx = [self.word_dict.get(sent[j], unk) if 0 <= j < len(sent) else unk
                       for j in range(vi - 2, vi + 3)]
                mark = [1 if abs(i - vi) <= 2 else 0 for i in range(len(sent))]
                n = len(sent)
                self.samples.append((wid, *[[c] * n for c in ctx],
                                     [self.predicate_dict.get(sent[vi], 0)] * n, mark,
                                     [self.label_dict.get(t, 0) for t in tags]))

    def __getitem__(self, idx):
        return tuple(np.array(x) for x in self.samples[idx])

    def __len__(self):
        return len(self.samples)

    def get_dict(self):
        return self.word_dict, self.predicate_dict, self.label_dict

    def get_embedding(self):
        return self.emb_file


__all__ = ['Conll05st', 'Imdb', 'Imikolov', 'Movielens', 'UCIHousing', 'WMT14', 'WMT16']
