// ORACLE -- test infrastructure / CPU baseline only; never part of the product path.
//
// Faithful C++ restatement of the reference pipeline (/root/reference/src/main.rs),
// timed by bench.py as the CPU baseline ("kind": "port").  Structure kept:
//   split_file   main.rs:36-51   read lines, validate UTF-8, deal line i to chunk i%8
//   map_phase    main.rs:53-92   8 workers pop chunk indices from a mutex queue; each
//                                worker clones all chunks first (chunks.to_vec(), :62)
//   count_words  main.rs:94-101  split_whitespace + to_lowercase + HashMap += 1
//   write_map_result :103-109    one "word count\n" write(2) per entry (the reference
//                                does one tokio write_all per line)
//   reduce_phase main.rs:111-150 4 workers pop file names, parse, merge under ONE mutex
//   read_map_result :152-168     lines with exactly 2 whitespace fields, usize count
//   write_final_result :170-182  final_result.txt "word count\n" (we truncate on open;
//                                the reference does not -- SURVEY.md §0.2 quirk)
//   print_top_words :184-192     "Top 10 words:" + "word: count", stable sort by count desc
//   cleanup :194-202             delete map files, "Successfully deleted: <name>"
// Semantics of tokens/case come from the oracle restatement (mox_oracle.c).
// PARITY UNPINNED (see mox_oracle.c).
//
// Usage: meduce_ref [path=shakes.txt] [--workdir DIR] [--quiet] [--time]
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <iostream>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mox_oracle.h"

using Map = std::unordered_map<std::string, size_t>;

static bool decode_ws_at(const std::string& s, size_t i, size_t* len) {
  unsigned char c = (unsigned char)s[i];
  uint32_t cp;
  if (c < 0x80) { cp = c; *len = 1; }
  else if (c < 0xE0) { cp = ((c & 0x1F) << 6) | (s[i + 1] & 0x3F); *len = 2; }
  else if (c < 0xF0) { cp = ((c & 0x0F) << 12) | ((s[i + 1] & 0x3F) << 6) | (s[i + 2] & 0x3F); *len = 3; }
  else { cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3F) << 12) | ((s[i + 2] & 0x3F) << 6) | (s[i + 3] & 0x3F); *len = 4; }
  return moxo_is_whitespace(cp) != 0;
}

// str::split_whitespace
template <class F>
static void split_whitespace(const std::string& s, F&& f) {
  size_t i = 0, n = s.size(), cl;
  while (i < n) {
    if (decode_ws_at(s, i, &cl)) { i += cl; continue; }
    size_t st = i;
    while (i < n && !decode_ws_at(s, i, &cl)) i += cl;
    f(st, i - st);
  }
}

static Map count_words(const std::string& text) {  // main.rs:94-101
  Map m;
  std::string buf;
  split_whitespace(text, [&](size_t st, size_t len) {
    buf.resize(len * 2 + 8);
    size_t l = moxo_lowercase((const uint8_t*)text.data() + st, len, (uint8_t*)&buf[0]);
    m[std::string(buf.data(), l)] += 1;
  });
  return m;
}

static std::string g_dir = ".";

static void write_map_result(const std::string& name, const Map& m) {  // :103-109
  std::string path = g_dir + "/" + name;
  int fd = open(path.c_str(), O_WRONLY | O_CREAT | O_TRUNC, 0644);
  if (fd < 0) { perror(path.c_str()); exit(1); }
  char line[64];
  for (auto& kv : m) {
    std::string s = kv.first;
    snprintf(line, sizeof line, " %zu\n", kv.second);
    s += line;
    if (write(fd, s.data(), s.size()) != (ssize_t)s.size()) { perror("write"); exit(1); }
  }
  close(fd);
}

static Map read_map_result(const std::string& name) {  // :152-168
  std::ifstream in(g_dir + "/" + name, std::ios::binary);
  Map m;
  std::string line;
  while (std::getline(in, line)) {
    if (!line.empty() && line.back() == '\r') line.pop_back();
    std::vector<std::pair<size_t, size_t>> parts;
    split_whitespace(line, [&](size_t st, size_t len) { parts.emplace_back(st, len); });
    if (parts.size() == 2) {
      // parts[1].parse::<usize>() (main.rs:161): an optional '+', then one or
      // more ASCII digits, no overflow of u64; anything else is skipped
      std::string num = line.substr(parts[1].first, parts[1].second);
      size_t k = (!num.empty() && num[0] == '+') ? 1 : 0;
      bool ok = num.size() > k;
      unsigned long long v = 0;
      for (size_t j = k; ok && j < num.size(); j++) {
        const char c = num[j];
        ok = c >= '0' && c <= '9' && v <= (~0ull - (unsigned)(c - '0')) / 10;
        if (ok) v = v * 10 + (unsigned)(c - '0');
      }
      if (ok) m[line.substr(parts[0].first, parts[0].second)] = v;
    }
  }
  return m;
}

int main(int argc, char** argv) {
  std::string path = "shakes.txt";
  bool quiet = false, timing = false;
  for (int i = 1; i < argc; i++) {
    std::string a = argv[i];
    if (a == "--workdir" && i + 1 < argc) g_dir = argv[++i];
    else if (a == "--quiet") quiet = true;
    else if (a == "--time") timing = true;
    else path = a;
  }
  const int num_map_workers = 8, num_reduce_workers = 4, num_chunks = 8;  // main.rs:11-13
  auto t0 = std::chrono::steady_clock::now();

  // split_file (main.rs:36-51)
  std::string data;
  {
    std::ifstream in(path, std::ios::binary);
    if (!in) { std::cerr << "Error: cannot open " << path << "\n"; return 1; }
    std::ostringstream ss;
    ss << in.rdbuf();
    data = ss.str();
  }
  if (moxo_utf8_invalid_at((const uint8_t*)data.data(), data.size()) >= 0) {
    std::cerr << "Error: stream did not contain valid UTF-8\n";
    return 1;
  }
  std::vector<std::string> chunks(num_chunks);
  {
    size_t i = 0, n = data.size();
    int ci = 0;
    while (i < n) {
      size_t e = data.find('\n', i);
      size_t le = (e == std::string::npos) ? n : e;
      size_t ll = le - i;
      if (ll > 0 && data[le - 1] == '\r' && e != std::string::npos) ll--;
      chunks[ci].append(data, i, ll);
      chunks[ci].push_back('\n');
      ci = (ci + 1) % num_chunks;
      i = (e == std::string::npos) ? n : e + 1;
    }
  }
  data.clear();
  data.shrink_to_fit();
  auto t1 = std::chrono::steady_clock::now();

  // map_phase (main.rs:53-92)
  std::vector<int> queue;
  for (int i = 0; i < num_chunks; i++) queue.push_back(i);
  std::mutex qm, rm;
  std::vector<std::string> map_results;
  {
    std::vector<std::thread> th;
    for (int w = 0; w < num_map_workers; w++) {
      std::vector<std::string> mine = chunks;  // chunks.to_vec() (main.rs:62), on the spawning thread
      th.emplace_back([&, w, mine = std::move(mine)]() {
        for (;;) {
          int idx;
          {
            std::lock_guard<std::mutex> g(qm);
            if (queue.empty()) break;
            idx = queue.back();
            queue.pop_back();
          }
          Map counts = count_words(mine[idx]);
          std::string name = "map_" + std::to_string(w) + "_chunk_" + std::to_string(idx) + ".txt";
          write_map_result(name, counts);
          std::lock_guard<std::mutex> g(rm);
          map_results.push_back(name);
        }
      });
    }
    for (auto& t : th) t.join();
  }
  auto t2 = std::chrono::steady_clock::now();

  // reduce_phase (main.rs:111-150)
  Map final_result;
  {
    std::vector<std::string> rq = map_results;
    std::mutex fm;
    std::vector<std::thread> th;
    for (int w = 0; w < num_reduce_workers; w++) {
      th.emplace_back([&]() {
        for (;;) {
          std::string name;
          {
            std::lock_guard<std::mutex> g(qm);
            if (rq.empty()) break;
            name = rq.back();
            rq.pop_back();
          }
          Map wc = read_map_result(name);
          std::lock_guard<std::mutex> g(fm);  // one global lock for the whole merge (:131)
          for (auto& kv : wc) final_result[kv.first] += kv.second;
        }
      });
    }
    for (auto& t : th) t.join();
  }
  auto t3 = std::chrono::steady_clock::now();

  // write_final_result (main.rs:170-182)
  {
    std::string p = g_dir + "/final_result.txt";
    FILE* f = fopen(p.c_str(), "wb");
    if (!f) { perror(p.c_str()); return 1; }
    for (auto& kv : final_result) fprintf(f, "%s %zu\n", kv.first.c_str(), kv.second);
    fclose(f);
  }
  // print_top_words (main.rs:184-192)
  if (!quiet) {
    std::vector<std::pair<std::string, size_t>> v(final_result.begin(), final_result.end());
    std::stable_sort(v.begin(), v.end(), [](auto& a, auto& b) { return a.second > b.second; });
    printf("Top %d words:\n", 10);
    for (size_t i = 0; i < v.size() && i < 10; i++) printf("%s: %zu\n", v[i].first.c_str(), v[i].second);
  }
  // cleanup_intermediate_files (main.rs:194-202)
  for (auto& name : map_results) {
    std::string p = g_dir + "/" + name;
    if (unlink(p.c_str()) == 0) { if (!quiet) printf("Successfully deleted: %s\n", name.c_str()); }
    else fprintf(stderr, "Error deleting file %s: %s\n", name.c_str(), strerror(errno));
  }
  auto t4 = std::chrono::steady_clock::now();
  if (timing) {
    auto s = [](auto a, auto b) { return std::chrono::duration<double>(b - a).count(); };
    fprintf(stderr, "{\"split_s\": %.6f, \"map_s\": %.6f, \"reduce_s\": %.6f, \"hot_s\": %.6f, \"total_s\": %.6f, \"uniques\": %zu}\n",
            s(t0, t1), s(t1, t2), s(t2, t3), s(t0, t3), s(t0, t4), final_result.size());
  }
  return 0;
}
