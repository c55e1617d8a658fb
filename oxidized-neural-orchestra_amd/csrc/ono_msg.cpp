// ono_msg.cpp — what a ring worker's WorkerHandle::recv_event makes of a frame
// that is not the gradient it waits for (comms/src/handles/worker.rs:82-130,
// comms/src/protocol/msg.rs:160-191), so the TCP edge fails with the
// reference's error class and message:
//
//   kind 0  Msg::Control(serde_json::from_slice(payload)?)            msg.rs:171
//           malformed JSON / unknown command        -> the serde io::Error  (ONO_E_IO)
//           Upgraded, Disconnect, Done, ReportLoss  -> a WorkerEvent the ring
//               rejects: "Received an invalid worker event"               (ONO_E_PROTO)
//               (worker_ring.rs:136-138, 195-197)
//           ReportLoss holding a NaN (JSON null, msg.rs:201-229)
//                                                   -> "loss diverged: NaN or Inf detected"
//                                                      (worker.rs:110-115)              (ONO_E_IO)
//           any other command                       -> "Unexpected message from worker"
//                                                      (worker.rs:123-126)              (ONO_E_IO)
//   kind 5  Params, kind 6 Datachunk                -> "Unexpected message from worker" (ONO_E_IO)
//
// Command is an externally tagged serde enum with snake_case names
// (msg.rs:41-88): a unit command is the JSON string "done" (or {"done": null}),
// a struct command {"report_loss": {"losses": [...]}} (or its sequence form
// {"report_loss": [[...]]}).  The parser below is a strict JSON reader in
// serde_json's sense (no trailing commas or comments, no leading zeros,
// escapes checked, nesting limited to 128, nothing after the value but
// whitespace, numbers that overflow f64 rejected).  Only ReportLoss's payload
// is type-checked field by field; for the other struct commands the payload
// must be an object or array, its fields are not (they all end in "Unexpected
// message" when well formed).
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "ono_internal.h"

namespace ono {
namespace {

struct JVal {
    enum T { NUL, BOOL, NUM, STR, ARR, OBJ } t = NUL;
    double num = 0;
    std::string str;
    std::vector<JVal> arr;
    std::vector<std::pair<std::string, JVal>> obj;
};

class JsonReader {
public:
    JsonReader(const uint8_t *p, size_t n) : p_(p), n_(n) {}
    bool parse(JVal &v) {
        ws();
        if (!value(v, 0)) return false;
        ws();
        if (i_ != n_) return fail("trailing characters");
        return true;
    }
    std::string err;

private:
    bool fail(const char *what) {
        if (err.empty()) {
            char b[160];
            snprintf(b, sizeof b, "%s at byte %zu", what, i_);
            err = b;
        }
        return false;
    }
    void ws() {
        while (i_ < n_ && (p_[i_] == ' ' || p_[i_] == '\t' || p_[i_] == '\n' || p_[i_] == '\r')) i_++;
    }
    bool lit(const char *s) {
        size_t k = strlen(s);
        if (n_ - i_ < k || memcmp(p_ + i_, s, k) != 0) return fail("expected value");
        i_ += k;
        return true;
    }
    bool value(JVal &v, int depth) {
        if (depth > 127) return fail("recursion limit exceeded");
        if (i_ >= n_) return fail("EOF while parsing a value");
        switch (p_[i_]) {
        case 'n': v.t = JVal::NUL; return lit("null");
        case 't': v.t = JVal::BOOL; v.num = 1; return lit("true");
        case 'f': v.t = JVal::BOOL; v.num = 0; return lit("false");
        case '"': v.t = JVal::STR; return string(v.str);
        case '[': return array(v, depth);
        case '{': return object(v, depth);
        default:
            if (p_[i_] == '-' || (p_[i_] >= '0' && p_[i_] <= '9')) return number(v);
            return fail("expected value");
        }
    }
    bool digits() {
        size_t s = i_;
        while (i_ < n_ && p_[i_] >= '0' && p_[i_] <= '9') i_++;
        return i_ > s;
    }
    bool number(JVal &v) {
        const size_t s = i_;
        if (p_[i_] == '-') i_++;
        if (i_ >= n_) return fail("EOF while parsing a value");
        if (p_[i_] == '0') {
            i_++;
            if (i_ < n_ && p_[i_] >= '0' && p_[i_] <= '9') return fail("invalid number");
        } else if (!digits()) {
            return fail("invalid number");
        }
        if (i_ < n_ && p_[i_] == '.') {
            i_++;
            if (!digits()) return fail("invalid number");
        }
        if (i_ < n_ && (p_[i_] == 'e' || p_[i_] == 'E')) {
            i_++;
            if (i_ < n_ && (p_[i_] == '+' || p_[i_] == '-')) i_++;
            if (!digits()) return fail("invalid number");
        }
        std::string t(reinterpret_cast<const char *>(p_ + s), i_ - s);
        v.t = JVal::NUM;
        v.num = strtod(t.c_str(), nullptr);
        if (std::isinf(v.num)) return fail("number out of range");
        return true;
    }
    static void utf8(std::string &out, uint32_t c) {
        if (c < 0x80) {
            out += (char)c;
        } else if (c < 0x800) {
            out += (char)(0xC0 | (c >> 6));
            out += (char)(0x80 | (c & 0x3F));
        } else if (c < 0x10000) {
            out += (char)(0xE0 | (c >> 12));
            out += (char)(0x80 | ((c >> 6) & 0x3F));
            out += (char)(0x80 | (c & 0x3F));
        } else {
            out += (char)(0xF0 | (c >> 18));
            out += (char)(0x80 | ((c >> 12) & 0x3F));
            out += (char)(0x80 | ((c >> 6) & 0x3F));
            out += (char)(0x80 | (c & 0x3F));
        }
    }
    bool hex4(uint32_t &c) {
        if (n_ - i_ < 4) return fail("EOF while parsing a string");
        c = 0;
        for (int k = 0; k < 4; k++) {
            const uint8_t h = p_[i_++];
            c <<= 4;
            if (h >= '0' && h <= '9') c |= h - '0';
            else if (h >= 'a' && h <= 'f') c |= h - 'a' + 10;
            else if (h >= 'A' && h <= 'F') c |= h - 'A' + 10;
            else return fail("invalid escape");
        }
        return true;
    }
    // a UTF-8 sequence starting at p_[i_] (from_slice validates the bytes)
    bool utf8_seq(std::string &out) {
        const uint8_t b = p_[i_];
        int k = b >= 0xF0 && b <= 0xF4 ? 3 : b >= 0xE0 ? 2 : b >= 0xC2 && b < 0xE0 ? 1 : -1;
        if (k < 0 || n_ - i_ < (size_t)k + 1) return fail("invalid unicode code point");
        uint32_t c = b & (0x3F >> k);
        for (int q = 1; q <= k; q++) {
            if ((p_[i_ + q] & 0xC0) != 0x80) return fail("invalid unicode code point");
            c = (c << 6) | (p_[i_ + q] & 0x3F);
        }
        if ((k == 2 && (c < 0x800 || (c >= 0xD800 && c < 0xE000))) || (k == 3 && (c < 0x10000 || c > 0x10FFFF)))
            return fail("invalid unicode code point");
        out.append(reinterpret_cast<const char *>(p_ + i_), (size_t)k + 1);
        i_ += (size_t)k + 1;
        return true;
    }
    bool string(std::string &out) {
        i_++;  // opening quote
        for (;;) {
            if (i_ >= n_) return fail("EOF while parsing a string");
            const uint8_t c = p_[i_];
            if (c == '"') { i_++; return true; }
            if (c < 0x20) return fail("control character (\\u0000-\\u001F) found while parsing a string");
            if (c >= 0x80) {
                if (!utf8_seq(out)) return false;
                continue;
            }
            if (c != '\\') { out += (char)c; i_++; continue; }
            i_++;
            if (i_ >= n_) return fail("EOF while parsing a string");
            const uint8_t e = p_[i_++];
            switch (e) {
            case '"': out += '"'; break;
            case '\\': out += '\\'; break;
            case '/': out += '/'; break;
            case 'b': out += '\b'; break;
            case 'f': out += '\f'; break;
            case 'n': out += '\n'; break;
            case 'r': out += '\r'; break;
            case 't': out += '\t'; break;
            case 'u': {
                uint32_t u = 0;
                if (!hex4(u)) return false;
                if (u >= 0xDC00 && u < 0xE000) return fail("lone leading surrogate in hex escape");
                if (u >= 0xD800 && u < 0xDC00) {
                    uint32_t lo = 0;
                    if (n_ - i_ < 2 || p_[i_] != '\\' || p_[i_ + 1] != 'u') return fail("unexpected end of hex escape");
                    i_ += 2;
                    if (!hex4(lo)) return false;
                    if (lo < 0xDC00 || lo >= 0xE000) return fail("lone leading surrogate in hex escape");
                    u = 0x10000 + ((u - 0xD800) << 10) + (lo - 0xDC00);
                }
                utf8(out, u);
                break;
            }
            default: return fail("invalid escape");
            }
        }
    }
    bool array(JVal &v, int depth) {
        v.t = JVal::ARR;
        i_++;
        ws();
        if (i_ < n_ && p_[i_] == ']') { i_++; return true; }
        for (;;) {
            v.arr.emplace_back();
            ws();
            if (!value(v.arr.back(), depth + 1)) return false;
            ws();
            if (i_ >= n_) return fail("EOF while parsing a list");
            if (p_[i_] == ',') { i_++; ws(); if (i_ < n_ && p_[i_] == ']') return fail("trailing comma"); continue; }
            if (p_[i_] == ']') { i_++; return true; }
            return fail("expected `,` or `]`");
        }
    }
    bool object(JVal &v, int depth) {
        v.t = JVal::OBJ;
        i_++;
        ws();
        if (i_ < n_ && p_[i_] == '}') { i_++; return true; }
        for (;;) {
            ws();
            if (i_ >= n_) return fail("EOF while parsing an object");
            if (p_[i_] != '"') return fail("key must be a string");
            v.obj.emplace_back();
            if (!string(v.obj.back().first)) return false;
            ws();
            if (i_ >= n_ || p_[i_] != ':') return fail("expected `:`");
            i_++;
            ws();
            if (!value(v.obj.back().second, depth + 1)) return false;
            ws();
            if (i_ >= n_) return fail("EOF while parsing an object");
            if (p_[i_] == ',') { i_++; ws(); if (i_ < n_ && p_[i_] == '}') return fail("trailing comma"); continue; }
            if (p_[i_] == '}') { i_++; return true; }
            return fail("expected `,` or `}`");
        }
    }
    const uint8_t *p_;
    size_t n_, i_ = 0;
};

// Command's variants (msg.rs:44-88), serde snake_case names
const char *const kUnit[] = {"disconnect", "done", "eof", "ping", "pong", "request_params",
                             "share_dataset", "stop_after_epoch", "upgraded"};
const char *const kStruct[] = {"connect", "accept", "create_node", "report_loss", "share_dataset_size",
                               "stats_request", "stats_response", "switch", "upgrade"};

template <size_t N> bool one_of(const std::string &s, const char *const (&names)[N]) {
    for (const char *n : names)
        if (s == n) return true;
    return false;
}

int serde_err(const std::string &what) { return set_error(ONO_E_IO, "control message: %s", what.c_str()); }

int unexpected(const std::string &what) {
    return set_error(ONO_E_IO, "Unexpected message from worker, got: %s", what.c_str());
}

// a unit command the ring receives as a WorkerEvent (worker.rs:109-122)
int unit_command(const std::string &name) {
    if (name == "upgraded" || name == "disconnect" || name == "done")
        return set_error(ONO_E_PROTO, "Received an invalid worker event (control command %s)", name.c_str());
    return unexpected("Control(" + name + ")");
}

// ReportLoss { losses } (msg.rs:61-64, 194-229): a sequence of numbers or
// nulls (null -> NaN); recv_event rejects a non-finite loss (worker.rs:113-115)
int report_loss(const JVal &payload) {
    const JVal *losses = nullptr;
    if (payload.t == JVal::OBJ) {
        for (const auto &kv : payload.obj) {
            if (kv.first != "losses") continue;  // serde ignores unknown fields
            if (losses) return serde_err("duplicate field `losses`");
            losses = &kv.second;
        }
        if (!losses) return serde_err("missing field `losses`");
    } else if (payload.t == JVal::ARR) {  // a struct in its sequence form
        if (payload.arr.empty()) return serde_err("invalid length 0, expected struct variant Command::ReportLoss");
        if (payload.arr.size() > 1) return serde_err("trailing characters");
        losses = &payload.arr[0];
    } else {
        return serde_err("invalid type, expected struct variant Command::ReportLoss");
    }
    if (losses->t != JVal::ARR) return serde_err("invalid type, expected a sequence of float elements which may include nulls");
    bool finite = true;
    for (const JVal &l : losses->arr) {
        if (l.t == JVal::NUL) finite = false;
        else if (l.t != JVal::NUM) return serde_err("invalid type, expected f64");
    }
    if (!finite) return set_error(ONO_E_IO, "loss diverged: NaN or Inf detected");
    return set_error(ONO_E_PROTO, "Received an invalid worker event (control command report_loss)");
}

int control(const uint8_t *p, size_t n) {
    JsonReader rd(p, n);
    JVal v;
    if (!rd.parse(v)) return serde_err(rd.err);
    std::string name;
    const JVal *payload = nullptr;
    if (v.t == JVal::STR) {
        name = v.str;
    } else if (v.t == JVal::OBJ) {
        if (v.obj.size() != 1) return serde_err(v.obj.empty() ? "expected value" : "expected `}`");
        name = v.obj[0].first;
        payload = &v.obj[0].second;
    } else {
        return serde_err("invalid type, expected enum Command");
    }
    if (one_of(name, kUnit)) {
        if (payload && payload->t != JVal::NUL) return serde_err("invalid type, expected unit variant");
        return unit_command(name);
    }
    if (one_of(name, kStruct)) {
        if (!payload) return serde_err("invalid type: unit variant, expected struct variant");
        if (name == "report_loss") return report_loss(*payload);
        if (payload->t != JVal::OBJ && payload->t != JVal::ARR) return serde_err("invalid type, expected struct variant");
        return unexpected("Control(" + name + ")");
    }
    return serde_err("unknown variant `" + name + "`");
}

}  // namespace

int worker_event_check(uint32_t kind, const uint8_t *payload, size_t n) {
    switch (kind & 0xFFu) {  // Header::from_be_bytes(..) as u8 (msg.rs:168)
    case 0: return control(payload, n);
    case 1: case 2: case 3: case 4: return ONO_OK;
    case 5: return unexpected("Data(Params)");
    case 6: return unexpected("Data(Datachunk)");
    default: return set_error(ONO_E_IO, "Received an invalid kind byte %u", kind & 0xFFu);
    }
}

}  // namespace ono

extern "C" int ono_worker_event_check(uint32_t kind, const uint8_t *payload, size_t nbytes) {
    if (!payload && nbytes) return ono::set_error(ONO_E_ARG, "payload is NULL");
    static const uint8_t empty = 0;
    return ono::worker_event_check(kind, payload ? payload : &empty, nbytes);
}
