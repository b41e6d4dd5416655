// Test stand-in for orb_slam2/include/BoostArchiver.h (the fork's map
// save/load headers, which pull in Boost.Serialization).  Boost is not in this
// image, so this is a minimal archive with the same surface the fork's
// serialisation code uses -- boost::archive::binary_oarchive / binary_iarchive
// over a std::ostream / std::istream (no_header), `ar & x`, `oa << x`,
// `ia >> x`, boost::serialization::access as the friend that reaches private
// serialize() members -- and the behaviour the keyframe database relies on:
// pointers are tracked (an object reached twice is written once and loaded as
// one object; an object is registered before its members load, so pointer
// cycles such as KeyFrame -> KeyFrameDatabase -> KeyFrame resolve), and
// std::vector / std::list / std::map / std::set and DBoW2::BowVector are
// containers of their elements.  Test scaffolding only: a real build uses
// Boost through the fork's own header.
#pragma once
#include <cstdint>
#include <istream>
#include <list>
#include <map>
#include <ostream>
#include <set>
#include <stdexcept>
#include <type_traits>
#include <unordered_map>
#include <vector>

#include "Thirdparty/DBoW2/DBoW2/BowVector.h"

namespace boost {
namespace serialization {
class access {
public:
    template <class A, class T>
    static void serialize(A &ar, T &t, unsigned v) { t.serialize(ar, v); }
    template <class T>
    static T *construct() { return new T(); }
};
}  // namespace serialization

namespace archive {
enum flags { no_header = 1 };

namespace detail {
template <class T> struct is_seq : std::false_type {};
template <class T, class A> struct is_seq<std::vector<T, A>> : std::true_type {};
template <class T, class A> struct is_seq<std::list<T, A>> : std::true_type {};
template <class T> struct is_map : std::false_type {};
template <class K, class V, class C, class A> struct is_map<std::map<K, V, C, A>> : std::true_type {};
template <class T> struct is_set : std::false_type {};
template <class K, class C, class A> struct is_set<std::set<K, C, A>> : std::true_type {};
}  // namespace detail

class binary_oarchive {
public:
    explicit binary_oarchive(std::ostream &os, unsigned = 0) : os_(os) {}
    template <class T> binary_oarchive &operator<<(const T &t) { put(const_cast<T &>(t)); return *this; }
    template <class T> binary_oarchive &operator&(const T &t) { return *this << t; }

private:
    std::ostream &os_;
    std::unordered_map<const void *, uint32_t> ids_;

    void raw(const void *p, size_t n) {
        if (!os_.write(static_cast<const char *>(p), (std::streamsize)n)) throw std::runtime_error("archive write");
    }
    template <class T> void put(T &t) {
        if constexpr (std::is_arithmetic_v<T> || std::is_enum_v<T>) {
            raw(&t, sizeof(T));
        } else if constexpr (std::is_pointer_v<T>) {
            if (!t) { uint32_t z = 0; raw(&z, 4); return; }
            auto it = ids_.find(t);
            if (it != ids_.end()) { raw(&it->second, 4); return; }
            const uint32_t id = (uint32_t)ids_.size() + 1;
            ids_[t] = id;
            raw(&id, 4);
            put(*t);
        } else if constexpr (std::is_same_v<T, DBoW2::BowVector>) {
            put(static_cast<std::map<DBoW2::WordId, DBoW2::WordValue> &>(t));
        } else if constexpr (detail::is_seq<T>::value || detail::is_set<T>::value) {
            uint64_t n = t.size();
            raw(&n, 8);
            for (auto &x : t) put(const_cast<std::remove_const_t<std::remove_reference_t<decltype(x)>> &>(x));
        } else if constexpr (detail::is_map<T>::value) {
            uint64_t n = t.size();
            raw(&n, 8);
            for (auto &kv : t) {
                auto k = kv.first;
                put(k);
                put(kv.second);
            }
        } else {
            boost::serialization::access::serialize(*this, t, 0u);
        }
    }
};

class binary_iarchive {
public:
    explicit binary_iarchive(std::istream &is, unsigned = 0) : is_(is) {}
    template <class T> binary_iarchive &operator>>(T &t) { get(t); return *this; }
    template <class T> binary_iarchive &operator&(T &t) { return *this >> t; }

private:
    std::istream &is_;
    std::vector<void *> objs_;   // id - 1 -> object

    void raw(void *p, size_t n) {
        if (!is_.read(static_cast<char *>(p), (std::streamsize)n)) throw std::runtime_error("archive read");
    }
    template <class T> void get(T &t) {
        if constexpr (std::is_arithmetic_v<T> || std::is_enum_v<T>) {
            raw(&t, sizeof(T));
        } else if constexpr (std::is_pointer_v<T>) {
            using O = std::remove_pointer_t<T>;
            uint32_t id;
            raw(&id, 4);
            if (id == 0) { t = nullptr; return; }
            if (id <= objs_.size()) { t = static_cast<T>(objs_[id - 1]); return; }
            if (id != objs_.size() + 1) throw std::runtime_error("archive object id out of order");
            O *o = boost::serialization::access::construct<O>();
            objs_.push_back(o);   // registered before its members: cycles resolve to it
            t = o;
            get(*o);
        } else if constexpr (std::is_same_v<T, DBoW2::BowVector>) {
            get(static_cast<std::map<DBoW2::WordId, DBoW2::WordValue> &>(t));
        } else if constexpr (detail::is_seq<T>::value) {
            uint64_t n;
            raw(&n, 8);
            t.clear();
            for (uint64_t i = 0; i < n; ++i) {
                typename T::value_type x{};
                get(x);
                t.push_back(x);
            }
        } else if constexpr (detail::is_set<T>::value) {
            uint64_t n;
            raw(&n, 8);
            t.clear();
            for (uint64_t i = 0; i < n; ++i) {
                typename T::value_type x{};
                get(x);
                t.insert(x);
            }
        } else if constexpr (detail::is_map<T>::value) {
            uint64_t n;
            raw(&n, 8);
            t.clear();
            for (uint64_t i = 0; i < n; ++i) {
                typename T::key_type k{};
                typename T::mapped_type v{};
                get(k);
                get(v);
                t.emplace(k, v);
            }
        } else {
            boost::serialization::access::serialize(*this, t, 0u);
        }
    }
};
}  // namespace archive
}  // namespace boost
