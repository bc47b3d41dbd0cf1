"""Pure-Python restatement of LearnBasePlus.store_batch_stats
(learn_base.py:58-109) and the Board methods it calls (board.py:22-44,
245-262), line for line, on board.py's list-of-lists.

TEST INFRASTRUCTURE ONLY — the checker of subproc_amd.stats in tests/; the
product package never imports it.  The Slack post and the parameter-store
write (learn_base.py:110-120) are replaced by returning (key, payload).
Python 3 differences: ``i // 8`` for board.py:257's Py2 ``i / 8``, and the
set of params is joined in sorted order (subproc_amd.stats documents why).
"""
Empty, Black, White = 0, 1, 2  # board.py:3-7


class _Board:
    def __init__(self):  # board.py:22-27
        self.board = [[Empty for _ in range(8)] for _ in range(8)]
        self.board[3][3] = self.board[4][4] = White
        self.board[3][4] = self.board[4][3] = Black
        self.turn = Black
        self.nturn = 0

    def _count(self, color):  # board.py:29-41
        return sum(1 for y in range(8) for x in range(8) if self.board[y][x] == color)

    def n_black(self):
        return self._count(Black)

    def n_white(self):
        return self._count(White)

    @staticmethod
    def _turn_from_string(s):  # board.py:245-251
        return Black if s == 'O' else (White if s == 'X' else Empty)

    def deserialize(self, board_str, turn_str, nturn):  # board.py:253-262
        i = 0
        for s in board_str:
            self.board[i // 8][i % 8] = self._turn_from_string(s)
            i += 1
        self.turn = self._turn_from_string(turn_str)
        self.nturn = nturn


def store_batch_stats(books, reference_rule=True):
    """learn_base.py:58-109; reference_rule=False replaces line 77's
    ``white_discs > black_wins`` by ``white_discs > black_discs``."""
    black_wins = 0
    white_wins = 0
    disc_diff = []
    book_ids = []
    black_name = 'black'
    white_name = 'white'
    params = set()
    for book_id, book, meta in books:
        try:
            last_book = book[0]
            last_board = _Board()
            last_board.deserialize(last_book['book'], last_book['whosturn'], last_book['turn'])
            black_discs = last_board.n_black()
            white_discs = last_board.n_white()
            disc_diff.append(black_discs - white_discs)
            if black_discs > white_discs:
                black_wins += 1
            elif white_discs > (black_wins if reference_rule else black_discs):
                white_wins += 1
            book_ids.append(book_id)
            black_name = meta['proc_a']
            white_name = meta['proc_b']
            params.add(meta['hamletparam'])
        except Exception:
            pass
    black_win_rate = float(black_wins) / float(len(books))
    white_win_rate = float(white_wins) / float(len(books))
    payload = {
        black_name + '_win_rate': black_win_rate,
        white_name + '_win_rate': white_win_rate,
        'min_disc_diff': min(disc_diff),
        'max_disc_diff': max(disc_diff),
        'avg_disc_diff': float(sum(disc_diff)) / float(len(books)),
        'params_used': ' / '.join(sorted(params)),
        'diffs': sorted(disc_diff),
    }
    return ['stats', str(min(book_ids)), str(max(book_ids))], payload
