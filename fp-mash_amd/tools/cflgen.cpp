// cflgen — synthetic CFL k-finger text at C3 scale (5,000 x 2 kb -> 10 M lines).
//
// Same output as fpmash.datagen.cfl_text (lyn2vec `--type basic --type_factorization CFL`,
// fingerprint_utils.py:95-110, 443-476; Duval, factorizations.py:102-126), which is pinned
// byte for byte against the fork's DNA1-CFL.txt; the Python version takes ~47 ms per 2 kb
// sequence, this one a few hundred microseconds.  Test tooling only (tests/test_cli.py checks
// it against datagen); not part of libfpmash.
//
// stdin: one record per line, "<id>\t<sequence>".  stdout: for every record and every cyclic
// window start (one window of the whole sequence when it is shorter than the window):
// "G00000<id>_0 l1 l2 ...\n", the Lyndon factor lengths of the upper-cased window.
#include <algorithm>
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

static void duval(const char *w, int n, std::string &out) {
    int k = 0;
    char num[16];
    while (k < n) {
        int i = k, j = k + 1;
        while (j < n && (unsigned char)w[i] <= (unsigned char)w[j]) {
            i = ((unsigned char)w[i] < (unsigned char)w[j]) ? k : i + 1;
            ++j;
        }
        while (k <= i) {
            int len = j - i;
            int m = snprintf(num, sizeof num, " %d", len);
            out.append(num, m);
            k += len;
        }
    }
}

static void record(const std::string &id, std::string seq, int window, std::string &out) {
    for (auto &c : seq) c = (char)toupper((unsigned char)c);
    const std::string head = "G00000" + id + "_0";
    if ((int)seq.size() < window) {
        out += head;
        duval(seq.data(), (int)seq.size(), out);
        out += '\n';
        return;
    }
    std::string ss = seq + seq.substr(0, window);
    for (size_t i = 0; i < seq.size(); ++i) {
        out += head;
        duval(ss.data() + i, window, out);
        out += '\n';
    }
}

int main(int argc, char **argv) {
    int window = argc > 1 ? atoi(argv[1]) : 100;
    int threads = argc > 2 ? atoi(argv[2]) : (int)std::max(1u, std::thread::hardware_concurrency());
    std::ios::sync_with_stdio(false);
    std::vector<std::string> ids, seqs;
    std::string line;
    while (std::getline(std::cin, line)) {
        size_t t = line.find('\t');
        if (t == std::string::npos) continue;
        ids.push_back(line.substr(0, t));
        seqs.push_back(line.substr(t + 1));
    }
    const size_t n = seqs.size();
    std::vector<std::string> out(n);
    threads = std::max(1, std::min<int>(threads, 64));
    std::vector<std::thread> pool;
    for (int t = 0; t < threads; ++t)
        pool.emplace_back([&, t] {
            for (size_t r = t; r < n; r += threads) record(ids[r], seqs[r], window, out[r]);
        });
    for (auto &th : pool) th.join();
    for (auto &o : out) fwrite(o.data(), 1, o.size(), stdout);
    return 0;
}
