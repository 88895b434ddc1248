// kmhg_fastx.h -- host FASTA/FASTQ record reader for count.kmers.fq.sh.rp (plain or gzip, via
// zlib's gzread, as the reference reads it: src/kmer_reader.c:41-76).
//
// Record semantics follow the kseq parser the reference bundles (src/kseq.h, kseq_read):
//   * a record starts at the next '>' or '@' (anything before is skipped); the name runs to the
//     first isspace() char, a comment to the end of that line
//   * sequence lines follow until a line starting with '>', '+' or '@' (empty lines skipped);
//     after every line a trailing '\r' of the accumulated string is dropped (when it holds > 1
//     char) -- the same rule strips the quality lines
//   * '+' starts the quality: the rest of the '+' line is skipped (EOF there: error -2), then
//     whole lines are appended (at least one) until the quality is at least as long as the
//     sequence; a length mismatch is error -2
//   * read() returns the sequence length, -1 at end of file, -2 on a quality error; has_qual is
//     false for a FASTA record
// kmer_reader_read stops at the first negative return and after max_reads records.
#pragma once
#include <zlib.h>

#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

namespace kmhg {

class FastxReader {
 public:
  explicit FastxReader(const char* path) : gz_(gzopen(path, "rb")), buf_(1 << 20) {
    if (gz_) gzbuffer(gz_, 1 << 20);
  }
  ~FastxReader() { if (gz_) gzclose(gz_); }
  FastxReader(const FastxReader&) = delete;
  FastxReader& operator=(const FastxReader&) = delete;
  bool ok() const { return gz_ != nullptr; }

  int read(std::string& seq, std::string& qual, bool& has_qual) {
    int c;
    seq.clear();
    qual.clear();
    has_qual = false;
    if (last_ == 0) {                                   // jump to the next header
      while ((c = getc()) >= 0 && c != '>' && c != '@') {}
      if (c < 0) return -1;
      last_ = c;
    }
    // name: up to the first isspace(); EOF with nothing read ends the file
    int delim = 0;
    bool got = false;
    while ((c = getc()) >= 0) {
      got = true;
      if (is_space(c)) { delim = c; break; }
    }
    if (c < 0 && !got) return -1;
    if (delim != '\n') skip_line();                     // comment
    while ((c = getc()) >= 0 && c != '>' && c != '+' && c != '@') {
      if (c == '\n') continue;
      seq.push_back((char)c);
      append_line(seq);
    }
    if (c == '>' || c == '@') last_ = c;
    if (c != '+') { last_ = (c == '>' || c == '@') ? c : 0; return (int)seq.size(); }
    while ((c = getc()) >= 0 && c != '\n') {}           // rest of the '+' line
    if (c < 0) return -2;
    // kseq reads one quality line before it compares lengths (so even for an empty sequence)
    while (append_line(qual) && qual.size() < seq.size()) {}
    last_ = 0;
    if (qual.size() != seq.size()) return -2;
    has_qual = true;
    return (int)seq.size();
  }

 private:
  static bool is_space(int c) {
    return c == ' ' || c == '\t' || c == '\n' || c == '\v' || c == '\f' || c == '\r';
  }
  int getc() {
    if (pos_ >= end_) {
      if (eof_) return -1;
      const int n = gzread(gz_, buf_.data(), (unsigned)buf_.size());
      if (n <= 0) { eof_ = true; return -1; }
      pos_ = 0;
      end_ = n;
    }
    return buf_[pos_++];
  }
  void skip_line() {
    int c;
    while ((c = getc()) >= 0 && c != '\n') {}
  }
  // rest of the line appended (the '\n' consumed); false when EOF came before any byte
  bool append_line(std::string& s) {
    bool got = false;
    for (;;) {
      if (pos_ >= end_) {
        if (eof_) break;
        const int n = gzread(gz_, buf_.data(), (unsigned)buf_.size());
        if (n <= 0) { eof_ = true; break; }
        pos_ = 0;
        end_ = n;
      }
      got = true;
      const unsigned char* b = buf_.data() + pos_;
      const void* nl = memchr(b, '\n', (size_t)(end_ - pos_));
      const int take = nl ? (int)((const unsigned char*)nl - b) : end_ - pos_;
      s.append((const char*)b, (size_t)take);
      pos_ += take;
      if (nl) { ++pos_; break; }
    }
    if (!got) return false;
    if (s.size() > 1 && s.back() == '\r') s.pop_back();
    return true;
  }

  gzFile gz_;
  std::vector<unsigned char> buf_;
  int pos_ = 0, end_ = 0;
  bool eof_ = false;
  int last_ = 0;
};

}  // namespace kmhg
