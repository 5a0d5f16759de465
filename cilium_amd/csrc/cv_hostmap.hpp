// cv_hostmap.hpp — host-side store of a BPF map with the kernel's semantics
// (kernel/bpf/hashtab.c, lpm_trie.c as used through pkg/bpf/bpf.go:101-245).
//
// This is the authoritative copy of every map the agent writes; the device tables
// are compiled from it (cv_ctx.cpp).  HASH / LRU_HASH / PERCPU_HASH: exact match on
// the key bytes.  LPM_TRIE: an element is identified by (prefixlen, first prefixlen
// bits of the data); lookup is longest-prefix; the stored data bytes are the last
// ones written (host bits included, as the kernel keeps them).
#pragma once
#include <errno.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <memory>
#include <vector>

namespace cv {

// open-addressing byte-key table with tombstones
class ByteTable {
  public:
    ByteTable(uint32_t ks, uint32_t vs) : ks_(ks), vs_(vs) { rehash(16); }

    uint32_t size() const { return count_; }
    uint32_t capacity() const { return cap_; }
    uint32_t ks() const { return ks_; }
    uint32_t vs() const { return vs_; }

    int64_t find(const uint8_t *k) const
    {
        uint64_t m = cap_ - 1, i = hash(k) & m;
        for (;;) {
            uint8_t st = state_[i];
            if (st == 0) return -1;
            if (st == 2 && !memcmp(&keys_[i * ks_], k, ks_)) return (int64_t)i;
            i = (i + 1) & m;
        }
    }
    // insert a new key (caller checked absence); returns slot
    int64_t insert(const uint8_t *k)
    {
        if ((count_ + dead_ + 1) * 4 > cap_ * 3) rehash(count_ * 2 + 16 > cap_ ? cap_ * 2 : cap_);
        uint64_t m = cap_ - 1, i = hash(k) & m;
        while (state_[i] == 2) i = (i + 1) & m;
        if (state_[i] == 1) dead_--;
        state_[i] = 2;
        memcpy(&keys_[i * ks_], k, ks_);
        memset(&vals_[i * vs_], 0, vs_);
        count_++;
        return (int64_t)i;
    }
    void erase(int64_t s)
    {
        state_[s] = 1;
        count_--;
        dead_++;
    }
    bool used(uint64_t s) const { return state_[s] == 2; }
    const uint8_t *key(uint64_t s) const { return &keys_[s * ks_]; }
    uint8_t *val(uint64_t s) { return &vals_[s * vs_]; }
    const uint8_t *val(uint64_t s) const { return &vals_[s * vs_]; }

  private:
    uint64_t hash(const uint8_t *k) const
    {
        uint64_t h = 0x84222325CBF29CE4ULL;
        for (uint32_t i = 0; i < ks_; ++i) h = (h ^ k[i]) * 0x100000001B3ULL;
        h ^= h >> 29; h *= 0xBF58476D1CE4E5B9ULL; h ^= h >> 32;
        return h;
    }
    void rehash(uint64_t ncap)
    {
        std::vector<uint8_t> ok, ov, os;
        ok.swap(keys_); ov.swap(vals_); os.swap(state_);
        uint64_t oc = cap_;
        cap_ = ncap; count_ = 0; dead_ = 0;
        keys_.assign(cap_ * ks_, 0); vals_.assign(cap_ * (vs_ ? vs_ : 1), 0); state_.assign(cap_, 0);
        for (uint64_t i = 0; i < oc; ++i) {
            if (os[i] != 2) continue;
            int64_t s = insert(&ok[i * ks_]);
            memcpy(&vals_[s * vs_], &ov[i * vs_], vs_);
        }
    }
    uint32_t ks_, vs_;
    uint64_t cap_ = 0;
    uint32_t count_ = 0, dead_ = 0;
    std::vector<uint8_t> keys_, vals_, state_;
};

class HostMap {
  public:
    int type;
    uint32_t ks, vs, max_entries, flags;
    uint64_t version = 1;      // bumped on every successful write
    // keys written or deleted since the consumer last compiled the map (LPM keys
    // masked to their prefix length); `log_full` once more than LOG_MAX were noted
    static constexpr size_t LOG_MAX = 4096;
    std::vector<std::vector<uint8_t>> log;
    bool log_full = false;
    void log_clear() { log.clear(); log_full = false; }

    HostMap(int type_, uint32_t ks_, uint32_t vs_, uint32_t max_, uint32_t flags_)
        : type(type_), ks(ks_), vs(vs_), max_entries(max_), flags(flags_)
    {
        if (is_lpm()) {
            dbits_ = (ks - 4) * 8;
            per_len_.reserve(dbits_ + 1);
            for (uint32_t l = 0; l <= dbits_; ++l) per_len_.emplace_back(ks - 4, ks - 4 + vs);
        } else {
            tab_.reset(new ByteTable(ks, vs));
        }
    }

    bool is_lpm() const { return type == 11; }

    // drop every element (a CT map whose device copy became authoritative)
    void clear()
    {
        if (is_lpm()) return;
        tab_.reset(new ByteTable(ks, vs));
        log_clear();
        version++;
    }
    uint32_t data_bits() const { return dbits_; }

    uint32_t count() const
    {
        if (!is_lpm()) return tab_->size();
        return lpm_count_;
    }

    int update(const uint8_t *key, const uint8_t *val, uint64_t fl)
    {
        if (fl > 2) return -EINVAL;
        if (is_lpm()) {
            uint32_t plen;
            memcpy(&plen, key, 4);
            if (plen > dbits_) return -EINVAL;
            std::vector<uint8_t> mk(key + 4, key + ks);
            mask(mk.data(), plen);
            ByteTable &t = per_len_[plen];
            int64_t s = t.find(mk.data());
            if (s >= 0) {
                if (fl == 1) return -EEXIST;
            } else {
                if (fl == 2) return -ENOENT;
                if (lpm_count_ >= max_entries) return -ENOSPC;
                s = t.insert(mk.data());
                lpm_count_++;
            }
            memcpy(t.val(s), key + 4, ks - 4);
            memcpy(t.val(s) + ks - 4, val, vs);
            version++;
            note(key, mk.data());
            return 0;
        }
        int64_t s = tab_->find(key);
        if (s >= 0) {
            if (fl == 1) return -EEXIST;
        } else {
            if (fl == 2) return -ENOENT;
            if (tab_->size() >= max_entries) return -E2BIG;
            s = tab_->insert(key);
        }
        memcpy(tab_->val(s), val, vs);
        version++;
        note(key, nullptr);
        return 0;
    }

    // value pointer of an exact element (HASH) / longest match (LPM), or null
    const uint8_t *lookup(const uint8_t *key) const
    {
        if (!is_lpm()) {
            int64_t s = tab_->find(key);
            return s >= 0 ? tab_->val(s) : nullptr;
        }
        uint32_t plen;
        memcpy(&plen, key, 4);
        if (plen > dbits_) plen = dbits_;
        std::vector<uint8_t> mk(ks - 4);
        for (int l = (int)plen; l >= 0; --l) {
            const ByteTable &t = per_len_[l];
            if (!t.size()) continue;
            memcpy(mk.data(), key + 4, ks - 4);
            mask(mk.data(), (uint32_t)l);
            int64_t s = t.find(mk.data());
            if (s >= 0) return t.val(s) + ks - 4;
        }
        return nullptr;
    }

    uint8_t *lookup_mut(const uint8_t *key) { return const_cast<uint8_t *>(lookup(key)); }

    int remove(const uint8_t *key)
    {
        if (!is_lpm()) {
            int64_t s = tab_->find(key);
            if (s < 0) return -ENOENT;
            tab_->erase(s);
            version++;
            note(key, nullptr);
            return 0;
        }
        uint32_t plen;
        memcpy(&plen, key, 4);
        if (plen > dbits_) return -ENOENT;
        std::vector<uint8_t> mk(key + 4, key + ks);
        mask(mk.data(), plen);
        int64_t s = per_len_[plen].find(mk.data());
        if (s < 0) return -ENOENT;
        per_len_[plen].erase(s);
        lpm_count_--;
        version++;
        note(key, mk.data());
        return 0;
    }

    // value of the exact element (LPM: same prefix length and masked prefix), or null
    const uint8_t *lookup_exact(const uint8_t *key) const
    {
        if (!is_lpm()) return lookup(key);
        uint32_t plen;
        memcpy(&plen, key, 4);
        if (plen > dbits_) return nullptr;
        std::vector<uint8_t> mk(key + 4, key + ks);
        mask(mk.data(), plen);
        const ByteTable &t = per_len_[plen];
        const int64_t s = t.find(mk.data());
        return s >= 0 ? t.val(s) + ks - 4 : nullptr;
    }

    // Walk every element: f(key bytes (BPF layout), value bytes).
    template <class F>
    void for_each(F f) const
    {
        if (!is_lpm()) {
            for (uint64_t s = 0; s < tab_->capacity(); ++s)
                if (tab_->used(s)) f(tab_->key(s), tab_->val(s));
            return;
        }
        std::vector<uint8_t> k(ks);
        for (uint32_t l = 0; l <= dbits_; ++l) {
            const ByteTable &t = per_len_[l];
            if (!t.size()) continue;
            for (uint64_t s = 0; s < t.capacity(); ++s) {
                if (!t.used(s)) continue;
                memcpy(k.data(), &l, 4);
                memcpy(k.data() + 4, t.val(s), ks - 4);
                f(k.data(), t.val(s) + ks - 4);
            }
        }
    }

    // GetNextKey: the element after `key` in walk order; the first one when key is
    // null or absent (kernel/bpf/hashtab.c htab_map_get_next_key).  -ENOENT at end.
    int next_key(const uint8_t *key, uint8_t *out) const
    {
        if (!is_lpm()) {                                  // the slot after key's, in table order
            uint64_t s = 0;
            if (key) {
                const int64_t at = tab_->find(key);
                s = at < 0 ? 0 : (uint64_t)at + 1;        // absent key: from the first element
            }
            for (; s < tab_->capacity(); ++s)
                if (tab_->used(s)) { memcpy(out, tab_->key(s), ks); return 0; }
            return -ENOENT;
        }
        bool take = key == nullptr, found = false, done = false;
        if (key && !exists_exact(key)) take = true;
        for_each([&](const uint8_t *k, const uint8_t *) {
            if (done) return;
            if (take) { memcpy(out, k, ks); done = true; return; }
            if (!memcmp(k, key, ks) || (is_lpm() && same_lpm_elem(k, key))) { take = true; found = true; }
        });
        (void)found;
        return done ? 0 : -ENOENT;
    }

    void note(const uint8_t *key, const uint8_t *masked)
    {
        if (log.size() >= LOG_MAX) { log_full = true; return; }
        std::vector<uint8_t> k(key, key + ks);
        if (masked) memcpy(k.data() + 4, masked, ks - 4);
        log.push_back(std::move(k));
    }

  private:
    bool exists_exact(const uint8_t *key) const
    {
        if (!is_lpm()) return tab_->find(key) >= 0;
        uint32_t plen;
        memcpy(&plen, key, 4);
        if (plen > dbits_) return false;
        std::vector<uint8_t> mk(key + 4, key + ks);
        mask(mk.data(), plen);
        return per_len_[plen].find(mk.data()) >= 0;
    }
    bool same_lpm_elem(const uint8_t *a, const uint8_t *b) const
    {
        if (memcmp(a, b, 4)) return false;
        uint32_t plen;
        memcpy(&plen, a, 4);
        std::vector<uint8_t> x(a + 4, a + ks), y(b + 4, b + ks);
        mask(x.data(), plen);
        mask(y.data(), plen);
        return x == y;
    }
    void mask(uint8_t *d, uint32_t plen) const
    {
        for (uint32_t b = 0; b < ks - 4; ++b) {
            uint32_t lo = b * 8;
            if (plen >= lo + 8) continue;
            d[b] = plen <= lo ? 0 : (uint8_t)(d[b] & (0xFF00u >> (plen - lo)));
        }
    }

    std::unique_ptr<ByteTable> tab_;
    std::vector<ByteTable> per_len_;
    uint32_t dbits_ = 0, lpm_count_ = 0;
};

}  // namespace cv
